"""Control plane of the aggregator: the two match tables of ngaa.p4 and the entries
bfrt/setup.py installs, as configuration for the device switch (ops.Switch) and its
egress (ops.route_ipv4), plus the bucket -> aggregator plan for several GPUs.

Reference (src/p4):
  switch_check   ngaa.p4:27-37   exact on hdr.ngaa.switch_id, size 1,
                                 actions set_agg / unset_agg, default unset_agg
  ipRoute        ngaa.p4:39-61   exact on hdr.ipv4.dst_addr, size 256,
                                 actions ipv4_forward(dst_addr: mac, port) / drop /
                                 NoAction, default drop
  entries        bfrt/setup.py:83-95  switch_check.add_with_set_agg(b'00000000') and
                                 three ipv4_forward rows (172.16.170.1-3 -> ports 132-134)

The bfrt shell names are kept (``cp.Ingress.switch_check.add_with_set_agg(0)``,
``add_with_ipv4_forward(dst_addr=..., dst_mac=..., port=...)``, ``dump``,
``clear_all``).  Two quirks of setup.py are accepted as it means them: it names the
route table ``ipv4_lpm`` (ngaa.p4 calls it ``ipRoute``; both names work here) and
writes the switch id as the bit string ``b'00000000'`` (read as binary, i.e. id 0).

The tables are host state (the Tofino's control plane is the bfrt shell on the
switch CPU); they reach the device as the Switch's switch_id and as the route
arrays ops.route_ipv4 stages in LDS.
"""
from __future__ import annotations

import ipaddress

import torch

from . import _lib, ops

PORT_DROP, PORT_NONE = _lib.PORT_DROP, _lib.PORT_NONE


def _switch_id_key(key) -> int:
    if isinstance(key, (bytes, bytearray)):
        key = key.decode()
    if isinstance(key, str):
        s = key.strip()
        key = int(s, 2) if s and set(s) <= {"0", "1"} else int(s, 0)
    key = int(key)
    if not 0 <= key <= 0xFF:
        raise ValueError(f"switch_id is bit<8> (headers.p4:35); got {key}")
    return key


def ip2int(ip) -> int:
    """IPv4 address (dotted string, ipaddress object or int) -> host-order int
    (setup.py:19-23's ip2int)."""
    if isinstance(ip, int):
        if not 0 <= ip <= 0xFFFFFFFF:
            raise ValueError(f"not an IPv4 address: {ip}")
        return ip
    return int(ipaddress.IPv4Address(str(ip) if not isinstance(ip, str) else ip.strip()))


class Table:
    """One exact-match table: key -> (action, params), a size limit and a default."""

    def __init__(self, name: str, key_name: str, size: int, actions: dict, default: str,
                 key_fn):
        self.name, self.key_name, self.size = name, key_name, size
        self._actions = actions              # action -> tuple of parameter names
        self._default0 = default
        self.default_action = default
        self._key_fn = key_fn
        self.entries: dict[int, tuple[str, dict]] = {}

    def _add(self, action: str, key, params: dict):
        k = self._key_fn(key)
        if k in self.entries:
            raise KeyError(f"{self.name}: entry for {self.key_name}={key!r} already exists")
        if len(self.entries) >= self.size:
            raise OverflowError(f"{self.name}: table full ({self.size} entries)")
        want = self._actions[action]
        missing = [p for p in want if p not in params]
        extra = [p for p in params if p not in want]
        if missing or extra:
            raise TypeError(f"{self.name}.{action}: parameters {want}, got {sorted(params)}")
        self.entries[k] = (action, dict(params))

    def __getattr__(self, attr):
        if attr.startswith("add_with_"):
            action = attr[len("add_with_"):]
            if action in self._actions:
                return lambda *a, **kw: self._add(action, *self._split(a, kw), self._params(kw))
        raise AttributeError(f"{self.name} has no attribute {attr}")

    def _split(self, args, kw):
        if args:
            return (args[0],)
        for k in (self.key_name, *self._aliases()):
            if k in kw:
                return (kw[k],)
        raise TypeError(f"{self.name}: missing key {self.key_name}")

    def _aliases(self):
        return ()

    def _params(self, kw):
        return {k: v for k, v in kw.items() if k not in (self.key_name, *self._aliases())}

    def delete(self, key):
        del self.entries[self._key_fn(key)]

    def get(self, key):
        return self.entries.get(self._key_fn(key), (self.default_action, {}))

    def clear(self):
        self.entries.clear()

    def reset_default(self):
        self.default_action = self._default0

    def dump(self, table: bool = True) -> list:
        rows = [(k, a, p) for k, (a, p) in sorted(self.entries.items())]
        if table:
            print(f"{self.name} ({len(rows)}/{self.size}, default {self.default_action})")
            for k, a, p in rows:
                print(f"  {self.key_name}={k:#x} -> {a}{p if p else ''}")
        return rows


class SwitchCheck(Table):
    """switch_check (ngaa.p4:27-37)."""

    def __init__(self):
        super().__init__("switch_check", "switch_id", 1, {"set_agg": (), "unset_agg": ()},
                         "unset_agg", _switch_id_key)

    def aggregating_id(self) -> int:
        """The switch_id whose packets are aggregated, or -1 when none is (an empty
        table or an unset_agg row: every NGA packet is 'other switches' job',
        ngaa.p4:184-186)."""
        for k, (a, _) in self.entries.items():
            if a == "set_agg":
                return k
        return -1


class IpRoute(Table):
    """ipRoute (ngaa.p4:39-61)."""

    def __init__(self):
        super().__init__("ipRoute", "dst_addr", 1 << 8,
                         {"ipv4_forward": ("dst_mac", "port"), "drop": (), "NoAction": ()},
                         "drop", ip2int)

    def _aliases(self):
        return ("dstAddr",)                 # setup.py:87 spelling

    def _params(self, kw):
        p = super()._params(kw)
        if "dstMacAddr" in p:               # setup.py:87 spelling of ipv4_forward's mac
            p["dst_mac"] = p.pop("dstMacAddr")
        return p

    def _add(self, action, key, params):
        if action == "ipv4_forward" and set(params) == {"dst_mac", "port"}:
            port = int(params["port"])
            if not 0 <= port < 512:
                raise ValueError(f"egress_spec_t is bit<9>; port {port}")
            params = {"dst_mac": int(params["dst_mac"]), "port": port}
        super()._add(action, key, params)

    def rows(self) -> list[tuple[int, int]]:
        """[(ipv4, port | PORT_DROP | PORT_NONE)] in insertion order."""
        out = []
        for k, (a, p) in self.entries.items():
            out.append((k, p["port"] if a == "ipv4_forward" else
                        PORT_DROP if a == "drop" else PORT_NONE))
        return out


class _Ingress:
    def __init__(self):
        self.switch_check = SwitchCheck()
        self.ipRoute = IpRoute()

    @property
    def ipv4_lpm(self):                     # the name setup.py:85 uses
        return self.ipRoute


class ControlPlane:
    """bfrt.nga.pipe for one aggregator: ``cp.Ingress.switch_check`` / ``cp.Ingress.ipRoute``."""

    def __init__(self):
        self.Ingress = _Ingress()

    def clear_all(self):
        for t in (self.Ingress.switch_check, self.Ingress.ipRoute):
            t.clear()
            t.reset_default()

    @property
    def switch_id(self) -> int:
        return self.Ingress.switch_check.aggregating_id()

    def route_table(self, device) -> tuple[torch.Tensor, torch.Tensor]:
        rows = self.Ingress.ipRoute.rows()
        keys = torch.tensor([k - (1 << 32) if k >= 1 << 31 else k for k, _ in rows],
                            dtype=torch.int32).to(device)
        ports = torch.tensor([p for _, p in rows], dtype=torch.int32).to(device)
        return keys, ports

    def make_switch(self, V: int, num_slots: int = _lib.NUM_REGISTER, device="cuda",
                    write_dropped: bool = False) -> ops.Switch:
        """A device switch whose switch_check is this table (-1 when it aggregates nothing)."""
        return ops.Switch(V, num_slots, self.switch_id, device, write_dropped)

    def egress(self, actions: torch.Tensor, dst_ip: torch.Tensor | None = None,
               dst_default=0) -> torch.Tensor:
        """ipRoute over a switched batch on the device (ops.route_ipv4)."""
        keys, ports = self.route_table(actions.device)
        return ops.route_ipv4(actions, keys, ports, dst_ip, ip2int(dst_default))


def reference_setup() -> ControlPlane:
    """The entries bfrt/setup.py:83-95 installs (switch 0 aggregates; three hosts)."""
    cp = ControlPlane()
    cp.clear_all()
    cp.Ingress.switch_check.add_with_set_agg(b"00000000")
    for ip, mac, port in (("172.16.170.1", 0x48DF37AAFAA8, 132),
                          ("172.16.170.2", 0x48DF375CFFB8, 133),
                          ("172.16.170.3", 0x48DF37AAACB8, 134)):
        cp.Ingress.ipv4_lpm.add_with_ipv4_forward(dstAddr=ipaddress.ip_address(ip),
                                                  dstMacAddr=mac, port=port)
    return cp


class BucketPlan:
    """Which aggregator owns which gradient bucket, and where its results go -- the
    switch_check/ipRoute configuration for several aggregators.

    Aggregator r (one GPU) answers to switch_id ``base_id + r``; buckets are assigned
    largest first to the least-loaded aggregator (LPT), so per-GPU bytes stay within
    one bucket of each other.  Worker packets for bucket b carry switch_id(b); an
    aggregator forwards other ids (ngaa.p4:184-186) to their owner's port and its own
    completed slots to the PS.
    """

    def __init__(self, bucket_values, n_aggregators: int, base_id: int = 1):
        if n_aggregators < 1 or base_id < 0 or base_id + n_aggregators - 1 > 0xFF:
            raise ValueError("switch ids are bit<8>: need 0 <= base_id, base_id + n - 1 <= 255")
        self.sizes = [int(v) for v in bucket_values]
        self.n, self.base_id = n_aggregators, base_id
        load = [0] * n_aggregators
        self.owner_of = [0] * len(self.sizes)
        for b in sorted(range(len(self.sizes)), key=lambda b: (-self.sizes[b], b)):
            r = min(range(n_aggregators), key=lambda r: (load[r], r))
            self.owner_of[b] = r
            load[r] += self.sizes[b]
        self.load = load

    def owner(self, bucket: int) -> int:
        return self.owner_of[bucket]

    def switch_id(self, bucket: int) -> int:
        return self.base_id + self.owner_of[bucket]

    def buckets_of(self, rank: int) -> list[int]:
        return [b for b, r in enumerate(self.owner_of) if r == rank]

    def control_plane(self, rank: int, ps_addr, ps_port: int, agg_addrs=(), agg_ports=()):
        """Aggregator `rank`'s tables: set_agg for its own id; ipRoute to the PS and to
        every other aggregator (agg_addrs[r] -> agg_ports[r])."""
        cp = ControlPlane()
        cp.Ingress.switch_check.add_with_set_agg(self.base_id + rank)
        cp.Ingress.ipRoute.add_with_ipv4_forward(ps_addr, dst_mac=0, port=ps_port)
        for r, (a, p) in enumerate(zip(agg_addrs, agg_ports)):
            if r != rank:
                cp.Ingress.ipRoute.add_with_ipv4_forward(a, dst_mac=0, port=p)
        return cp
