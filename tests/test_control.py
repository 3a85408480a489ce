"""Control plane (ina_amd.control): the switch_check / ipRoute tables of ngaa.p4:27-61
with the entries bfrt/setup.py:83-95 installs, the route restatement in the oracle,
and the bucket -> aggregator plan.  CPU only (table logic; no device calls)."""
import ipaddress

import numpy as np
import pytest
import torch

from ina_amd import control
from oracle import oracle as orc


def test_reference_setup_entries():
    cp = control.reference_setup()
    assert cp.switch_id == 0                              # b'00000000' read as bits
    rows = cp.Ingress.ipRoute.rows()
    assert rows == [(0xAC10AA01, 132), (0xAC10AA02, 133), (0xAC10AA03, 134)]
    assert cp.Ingress.ipv4_lpm is cp.Ingress.ipRoute      # setup.py's table name
    assert cp.Ingress.ipRoute.get("172.16.170.2") == ("ipv4_forward",
                                                      {"dst_mac": 0x48DF375CFFB8, "port": 133})
    assert cp.Ingress.ipRoute.get("10.0.0.1") == ("drop", {})     # default_action = drop


def test_switch_check_semantics():
    cp = control.ControlPlane()
    assert cp.switch_id == -1                             # default unset_agg
    cp.Ingress.switch_check.add_with_set_agg(7)
    assert cp.switch_id == 7
    with pytest.raises(OverflowError):                    # size = 1 (ngaa.p4:35)
        cp.Ingress.switch_check.add_with_set_agg(8)
    with pytest.raises(KeyError):
        cp.Ingress.switch_check.add_with_set_agg(7)
    cp.clear_all()
    cp.Ingress.switch_check.add_with_unset_agg(7)
    assert cp.switch_id == -1
    with pytest.raises(ValueError):
        control.ControlPlane().Ingress.switch_check.add_with_set_agg(256)
    assert control._switch_id_key("0x1f") == 31 and control._switch_id_key(b"101") == 5


def test_ip_route_table_limits_and_actions():
    cp = control.ControlPlane()
    t = cp.Ingress.ipRoute
    for i in range(256):
        t.add_with_ipv4_forward(f"10.0.{i // 256}.{i % 256}", dst_mac=i, port=i % 300)
    with pytest.raises(OverflowError):                    # size = 1<<8 (ngaa.p4:59)
        t.add_with_drop("10.1.0.0")
    t.delete("10.0.0.5")
    t.add_with_drop("10.1.0.0")
    with pytest.raises(ValueError):
        control.ControlPlane().Ingress.ipRoute.add_with_ipv4_forward("1.2.3.4", dst_mac=0, port=512)
    with pytest.raises(TypeError):
        control.ControlPlane().Ingress.ipRoute.add_with_ipv4_forward("1.2.3.4", port=1)
    cp2 = control.ControlPlane()
    cp2.Ingress.ipRoute.add_with_NoAction(ipaddress.ip_address("1.2.3.4"))
    cp2.Ingress.ipRoute.add_with_drop(dst_addr=0x01020305)
    assert cp2.Ingress.ipRoute.rows() == [(0x01020304, control.PORT_NONE),
                                         (0x01020305, control.PORT_DROP)]
    assert len(cp2.Ingress.ipRoute.dump(table=False)) == 2


def test_route_table_tensor_encoding():
    cp = control.reference_setup()
    cp.Ingress.ipRoute.add_with_drop("255.255.255.255")
    keys, ports = cp.route_table("cpu")
    assert keys.dtype == torch.int32 and ports.dtype == torch.int32
    assert keys.numpy().view(np.uint32).tolist() == [0xAC10AA01, 0xAC10AA02, 0xAC10AA03, 0xFFFFFFFF]
    assert ports.tolist() == [132, 133, 134, -1]


def test_device_route_refuses_cpu_tensors():
    from ina_amd import ops
    a = torch.zeros(4, dtype=torch.uint8)
    k = torch.zeros(1, dtype=torch.int32)
    with pytest.raises(ValueError):
        ops.route_ipv4(a, k, k)


def test_oracle_route_restatement():
    """ngaa.p4:120-196: every forwarded packet meets ipRoute; ingress drops never do."""
    act = np.array([orc.ACT_DROP, orc.ACT_FWD_AGG, orc.ACT_FWD_COLLISION, orc.ACT_FWD_ACK,
                    orc.ACT_FWD_OTHER, orc.ACT_FWD_AGG, orc.ACT_FWD_AGG], np.uint8)
    dst = np.array([1, 1, 2, 3, 1, 9, 3], np.uint32)
    table = [(1, 132), (2, orc.PORT_DROP), (3, orc.PORT_NONE), (1, 7)]   # first hit wins
    assert orc.route_ipv4(act, table, dst).tolist() == [-1, 132, -1, -2, 132, -1, -2]
    assert orc.route_ipv4(act, [], dst).tolist() == [-1] * 7              # default drop
    assert orc.route_ipv4(act, table, None, 1).tolist() == [-1] + [132] * 6


def test_bucket_plan_lpt_balance():
    sizes = [100, 90, 80, 70, 60, 50, 40, 30, 20, 10]
    plan = control.BucketPlan(sizes, 3, base_id=4)
    assert sorted(b for r in range(3) for b in plan.buckets_of(r)) == list(range(10))
    assert max(plan.load) - min(plan.load) <= max(sizes)
    assert sum(plan.load) == sum(sizes)
    assert {plan.switch_id(b) for b in range(10)} == {4, 5, 6}
    assert plan.owner(0) == 0 and plan.owner(1) == 1 and plan.owner(2) == 2   # LPT order
    cp = plan.control_plane(1, "10.0.0.100", 7, agg_addrs=["10.0.0.1", "10.0.0.2", "10.0.0.3"],
                            agg_ports=[11, 12, 13])
    assert cp.switch_id == 5
    assert dict(cp.Ingress.ipRoute.rows()) == {0x0A000064: 7, 0x0A000001: 11, 0x0A000003: 13}
    with pytest.raises(ValueError):
        control.BucketPlan([1], 2, base_id=255)
