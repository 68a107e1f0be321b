"""bench.measure_group_ingest's placement and split with 8 members on 8 distinct (fake)
devices, on the CPU: the N = 8 path that only the driver's 8-GPU node runs end to end.

bt_group is replaced by a recording stand-in (no HIP): it hands out one placement per member
(member k on device k, NUMA node k % 2), records every registration, and in run_mapped resolves
each member's byte range of the batch against the registrations and takes that member's alias
with "its device current" — the fake alias of device d is ((d + 1) << 48) + host address, as in
tests/cpp/test_pin.cpp's driver, whose eight_members case checks the same thing on the real
page table (bt_pin.h). NUMA binding is recorded instead of applied (the container has one node).
"""
import ctypes

import numpy as np
import pytest

import bench
from beatrice_amd import abi, numa, synth

N_DEV = 8
PACKETS = 8192
COST = (64, 64, 32)


class FakeGroup:
    made = []

    def __init__(self, devices, host_chunk_packets=0, flags=0, host_threads=0):
        self.devices = list(devices)
        self.flags = flags
        self.registered = {}      # host address -> array
        self.unregistered = []
        self.set_device = []      # device made current, in call order
        self.aliases = []         # (member, device, host lo, alias)
        self.compiled = None
        self.closed = False
        FakeGroup.made.append(self)

    def compile(self, filters):
        self.compiled = list(filters)

    def cost(self, mapped, records, filters, desc_bytes=8):
        assert mapped and not records and filters
        return COST

    def placement(self, k):
        return {"numa_node": k % 2, "pinned_cpus": 1, "pool_threads": 1, "staging_node": -1,
                "device": self.devices[k]}

    def register(self, arr):
        assert arr.ctypes.data % abi.PAGE == 0, "every registered buffer starts a page of its own"
        self.registered[arr.ctypes.data] = arr

    def unregister(self, arr):
        self.unregistered.append(arr.ctypes.data)

    def close(self):
        self.closed = True

    def _owner(self, lo, hi):
        for a, arr in self.registered.items():
            if a <= lo and hi <= a + arr.nbytes:
                return arr
        raise AssertionError(f"[{lo:#x}, {hi:#x}) is in no registered buffer")

    def run_mapped(self, batch, outs):
        desc = np.ctypeslib.as_array(ctypes.cast(batch.desc, ctypes.POINTER(ctypes.c_uint64)), (batch.n,))
        self._owner(batch.desc, batch.desc + 8 * batch.n)
        lens = synth.desc_len(desc)
        bounds = abi.group_split(lens, len(self.devices), COST, plan=True)
        dec = self._owner(outs.decide, outs.decide + batch.n)
        ver = self._owner(outs.verdict, outs.verdict + 8 * ((batch.n + 63) // 64))
        spans = numa.member_byte_ranges(synth.desc_off(desc), lens, bounds)
        for k, ((plo, phi), (blo, bhi)) in enumerate(zip(bounds, spans)):
            if phi <= plo:
                continue
            dev = self.devices[k]
            self.set_device.append(dev)   # the member's calls run with its device current
            lo, hi = batch.base + blo, batch.base + bhi
            self._owner(lo, hi)
            self.aliases.append((k, dev, lo, ((dev + 1) << 48) + lo))
            dec[plo:phi] = np.where(np.arange(plo, phi) % 3 == 0, 0x40, 0)   # some drop, most pass
        bits = (dec[:batch.n] >> 6) == 0
        ver[:] = np.packbits(np.pad(bits, (0, ver.size * 64 - batch.n)), bitorder="little").view(np.uint64)

    def run_host(self, data, desc, records=True, filters=True, outs=None):
        n = len(desc)
        outs["decide"][:n] = np.where(np.arange(n) % 3 == 0, 0x40, 0)
        return {"decide": outs["decide"][:n]}


@pytest.fixture
def fake(monkeypatch):
    FakeGroup.made = []
    placed = []

    def place_ranges(arr, ranges, hugepages=False):
        placed.append(list(ranges))
        return abi.host_copy(arr)

    monkeypatch.setattr(abi, "Group", FakeGroup)
    monkeypatch.setattr(abi, "device_count", lambda: N_DEV)
    monkeypatch.setattr(numa, "place_ranges", place_ranges)
    return placed


def test_eight_members_on_eight_devices(fake):
    out = bench.measure_group_ingest(N_DEV, PACKETS, reps=1)
    assert out["n_devices"] == N_DEV and not out["members_share_one_device"]
    assert len(FakeGroup.made) == 2   # one group per config (c2, c3)
    for name, grp, ranges in zip(("c2", "c3"), FakeGroup.made, fake):
        assert grp.devices == list(range(N_DEV)) and grp.flags == 0
        assert grp.compiled == bench.C3_FILTERS
        # placement: one byte range per member, back to back over the batch, member k's on
        # member k's node
        assert len(ranges) == N_DEV
        assert [nd for _, _, nd in ranges] == [k % 2 for k in range(N_DEV)]
        assert ranges[0][0] == 0 and all(ranges[k][1] <= ranges[k + 1][0] for k in range(N_DEV - 1))
        assert all(hi > lo for lo, hi, _ in ranges), "every member gets frames at this size"
        # every member resolved its own range with its own device current (warm-up + 1 rep)
        per_call = [a for a in grp.aliases[:N_DEV]]
        assert [k for k, *_ in per_call] == list(range(N_DEV))
        for k, dev, lo, alias in per_call:
            assert dev == k and alias == ((k + 1) << 48) + lo
        assert grp.set_device[:N_DEV] == list(range(N_DEV))
        assert len(grp.aliases) == 2 * N_DEV
        # the four buffers registered are released again, the group closed
        assert len(grp.registered) == 4 and sorted(grp.unregistered) == sorted(grp.registered)
        assert grp.closed
        ent = out[name]
        assert ent["verdicts_match_decisions"]
        assert ent["member_nodes"] == [k % 2 for k in range(N_DEV)]
        assert [p["device"] for p in ent["placement"]] == list(range(N_DEV))
        assert abs(ent["pass_fraction"] - 2 / 3) < 0.01
    assert out["c3_host_gather"]["decisions_match_zero_copy"]
    assert "ring" not in out   # the ring stage is a one-device entry


def test_member_ranges_follow_the_group_split(fake):
    """The split the bench places by is the plan the group's mapped call uses: member k's
    byte range covers exactly the frames of its packet range."""
    raw, desc = synth.capture(synth.C3, PACKETS)
    lens, offs = synth.desc_len(desc), synth.desc_off(desc)
    bounds = abi.group_split(lens, N_DEV, COST, plan=True)
    assert bounds[0][0] == 0 and bounds[-1][1] == PACKETS
    assert all(bounds[k][1] == bounds[k + 1][0] for k in range(N_DEV - 1))
    spans = numa.member_byte_ranges(offs, lens, bounds)
    for (plo, phi), (blo, bhi) in zip(bounds, spans):
        assert blo == int(offs[plo]) and bhi == int(offs[phi - 1] + lens[phi - 1])
        assert np.all(offs[plo:phi] >= blo) and np.all(offs[plo:phi] + lens[plo:phi] <= bhi)
