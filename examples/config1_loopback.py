#!/usr/bin/env python3
"""BASELINE config 1 on one GPU host: ResNet-50 (torchvision layout, 1000-way head:
25,557,032 parameters = PARA_LEN, communicator.py:11), worker_num=2, loopback sockets,
the P4 aggregator replaced by the PS GPU's packet-stream switch (ina_amd.loopback).

CIFAR-100 cannot be downloaded here (datasets.py:116-124 uses download=True), so each
worker trains on synthetic CIFAR-100-shaped batches (3x32x32, 100 labels, seeded).
Prints per-epoch timings in the style of launch.py:233-242.

  python examples/config1_loopback.py [--epochs 3] [--local-steps 5] [--batch 64]
"""
import argparse
import os
import socket
import sys
import tempfile
import threading
import time

import torch
import torch.multiprocessing as mp
import torch.nn as nn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1, down=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, width * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(width * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = down

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        return self.relu(self.bn3(self.conv3(y)) + idt)


class ResNet50(nn.Module):
    """torchvision.models.resnet50() layout (models.py:18), written out: torchvision is
    not installed here."""

    def __init__(self, num_classes=1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        cin, layers = 64, []
        for width, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
            down = nn.Sequential(nn.Conv2d(cin, width * 4, 1, stride, bias=False),
                                 nn.BatchNorm2d(width * 4))
            blk = [Bottleneck(cin, width, stride, down)]
            cin = width * 4
            blk += [Bottleneck(cin, width) for _ in range(blocks - 1)]
            layers.append(nn.Sequential(*blk))
        self.layer1, self.layer2, self.layer3, self.layer4 = layers
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(2048, num_classes)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


ARGS = None


def train_step(model, idx, epoch):
    """local SGD steps on synthetic CIFAR-100-shaped data (launch.py:285-300)."""
    dev = next(model.parameters()).device
    opt = torch.optim.SGD(model.parameters(), lr=max(0.97 * 0.01, 0.001))
    g = torch.Generator(device=dev).manual_seed(100 * idx + epoch)
    model.train()
    for _ in range(ARGS.local_steps):
        x = torch.randn(ARGS.batch, 3, 32, 32, device=dev, generator=g)
        y = torch.randint(0, 100, (ARGS.batch,), device=dev, generator=g)
        loss = nn.functional.cross_entropy(model(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()


def _worker(idx, W, port, path, args):
    global ARGS
    ARGS = args
    sys.path.insert(0, os.path.join(REPO, "distributed-training-ina_amd"))
    from ina_amd.loopback import worker_serve
    worker_serve(idx, W, port, path, ResNet50, train_step)


def main():
    global ARGS
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--local-steps", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--V", type=int, default=256)
    ap.add_argument("--k", type=int, default=16)
    ARGS = args = ap.parse_args()
    from ina_amd.loopback import ps_serve
    torch.manual_seed(0)
    model = ResNet50().cuda()
    n = sum(p.numel() for p in model.parameters())
    print(f"Model resnet50: {n} paras, {n * 4 / 2**20:.1f} MB; workers={args.workers}, V={args.V}")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "switch.sock")

        def report(e, vec, t_agg, t_tot):
            print(f"Epoch: {e}, throughput = {args.workers * args.batch / t_tot:.1f} image/s, "
                  f"switch+aggregate => {t_agg:.3f} sec, total => {t_tot:.3f} sec", flush=True)
        th = threading.Thread(target=ps_serve, args=(model, args.workers, args.epochs, port, path),
                              kwargs=dict(k=args.k, V=args.V, on_epoch=report, timeout_ms=600000))
        th.start()
        time.sleep(1.0)
        ctx = mp.get_context("spawn")
        procs = [ctx.Process(target=_worker, args=(i, args.workers, port, path, args))
                 for i in range(args.workers)]
        for p in procs:
            p.start()
        th.join()
        for p in procs:
            p.join()
    rc = max(p.exitcode for p in procs)
    print("workers exit codes:", [p.exitcode for p in procs])
    sys.exit(rc)


if __name__ == "__main__":
    main()
