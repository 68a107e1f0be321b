"""CPU, world_size 2 and 4 over gloo: the multi-GPU batch split (beatrice_amd/shard.py).
Each rank takes its tile-aligned, byte-balanced shard with rebased descriptors (what
one GPU would receive), computes it with the oracle standing in for the device, and
the host-side merge must equal the whole-batch result. No data-path collective:
only the results are gathered for the check."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as ol
from beatrice_amd import shard, synth

FILTERS = [{"type": 1, "expr": "udp", "priority": 3}, {"type": 2, "expr": "10.0.0.0/8", "priority": 2},
           {"type": 3, "expr": "1000-2000", "priority": 1}]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, cfg, n, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data, desc = synth.capture(cfg, n)
    bounds = shard.shard_bounds(synth.desc_len(desc), world)
    lo, hi = bounds[rank]
    local, ldesc = shard.local_batch(data, desc, lo, hi)
    rec, dec, npass = ol.oracle_run(local, ldesc, hi - lo, FILTERS, threads=2)
    bits = ((dec >> 6) == 0)
    ver = np.packbits(np.pad(bits, (0, (-len(bits)) % 64)), bitorder="little").view(np.uint64)
    part = {"decide": dec, "verdict": ver, "pass_idx": np.nonzero(bits)[0].astype(np.uint32),
            "n_pass": npass, "records": rec}
    parts = [None] * world
    dist.all_gather_object(parts, part)
    if rank == 0:
        m = shard.merge(parts, bounds, n)
        rec_all, dec_all, np_all = ol.oracle_run(data, desc, n, FILTERS, threads=2)
        ok = (np.array_equal(m["records"], rec_all) and np.array_equal(m["decide"], dec_all)
              and m["n_pass"] == np_all and np.array_equal(m["pass_idx"], np.nonzero((dec_all >> 6) == 0)[0]))
        q.put((ok, bounds))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg,n,world", [(synth.C3, 30000, 2), (synth.C4, 10001, 2), (synth.C3, 20037, 4)])
def test_rank_split_matches_whole_batch(cfg, n, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, cfg, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok, bounds = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
    assert ok, bounds
    assert bounds[0][0] == 0 and bounds[-1][1] == n and all(lo % 64 == 0 for lo, _ in bounds)
    assert all(bounds[i][1] == bounds[i + 1][0] for i in range(world - 1))


def test_bounds_balance_bytes():
    _, desc = synth.capture(synth.C3, 100000)
    ln = synth.desc_len(desc)
    for w in (2, 4, 8):
        b = shard.shard_bounds(ln, w)
        cost = [int((np.minimum(ln[lo:hi], 128) + 104).sum()) for lo, hi in b]
        assert max(cost) / (sum(cost) / w) < 1.01
        assert all(lo % 64 == 0 for lo, _ in b)


@pytest.mark.parametrize("seed", range(6))
def test_native_group_split_equals_shard_bounds(seed):
    """bt_group_split (the in-process multi-device split, C++) restates shard.shard_bounds
    exactly: the same tile-aligned, byte-balanced ranges for any lengths and member count."""
    from beatrice_amd import abi
    rng = np.random.default_rng(seed)
    for n in (0, 1, 63, 64, 65, 1000, 20037, int(rng.integers(1, 300000))):
        lens = rng.choice([0, 14, 60, 64, 128, 512, 1500, 9000, 65535], size=n).astype(np.uint32)
        for parts in (1, 2, 3, 4, 7, 8):
            assert abi.group_split(lens, parts) == shard.shard_bounds(lens, parts), (n, parts)


def test_native_group_split_rejects_bad_arguments():
    from beatrice_amd import abi
    with pytest.raises(abi.BtError):
        abi.group_split(np.zeros(10, np.uint32), 0)


@pytest.mark.parametrize("seed", range(4))
def test_native_split_cost_equals_shard_bounds(seed):
    """bt_group_split_cost (every cost model the group uses) against shard.shard_bounds."""
    from beatrice_amd import abi
    rng = np.random.default_rng(100 + seed)
    models = [shard.DEFAULT_COST] + [shard.group_cost(m, r, f, d, sb) for m in (False, True) for r in (False, True)
                                     for f in (False, True) for d in (0, 8, 16) for sb in (32, 48, 112, 176)]
    models += [(int(rng.integers(1, 300)), int(rng.choice([1, 4, 16, 64])), int(rng.integers(0, 200)))
               for _ in range(8)]
    for n in (0, 1, 64, 65, 4097, int(rng.integers(1, 200000))):
        lens = rng.choice([0, 14, 42, 60, 64, 90, 128, 512, 1500, 9000], size=n).astype(np.uint32)
        for cost in models:
            for parts in (1, 2, 3, 8):
                assert abi.group_split(lens, parts, cost) == shard.shard_bounds(lens, parts, cost=cost), \
                    (n, parts, cost)


def test_split_cost_balances_what_the_call_moves():
    """A verdict-only host batch stages 32 B of each frame: with that model an IMIX batch's
    members stage equal bytes, where the old 128 + 104 model over-weighted long frames."""
    _, desc = synth.capture(synth.C3, 200000)
    ln = synth.desc_len(desc)
    model = shard.group_cost(False, False, True)
    for w in (2, 4, 8):
        b = shard.shard_bounds(ln, w, cost=model)
        staged = [int(shard.packet_cost(ln[lo:hi], model).sum()) for lo, hi in b]
        assert max(staged) / (sum(staged) / w) < 1.01
        old = shard.shard_bounds(ln, w)
        staged_old = [int(shard.packet_cost(ln[lo:hi], model).sum()) for lo, hi in old]
        assert max(staged) <= max(staged_old)


def test_thread_budget_matches_mirror():
    """bt_group_thread_budget: one host-thread budget per group, split across members."""
    from beatrice_amd import abi
    for members in range(1, 17):
        for usable in (1, 2, 8, 16, 64, 256):
            for requested in (0, 1, 4, 16, 64, 128):
                got = abi.group_thread_budget(members, usable, requested)
                assert got == shard.member_threads(members, usable, requested)
                assert 1 <= got <= 16
    assert shard.member_threads(1, 16) == 16       # one context: the single-context default
    assert shard.member_threads(2, 16) == 8
    assert shard.member_threads(8, 16) == 2        # 8 GPUs on a 16-CPU job: 16 threads in all
    assert shard.member_threads(8, 128) == 16
    with pytest.raises(abi.BtError):
        abi.group_thread_budget(0, 16, 0)


def test_node_cpus_are_this_process_cpus():
    """bt_node_cpus: a NUMA node's CPUs this process may run on (the pool workers' pin set)."""
    from beatrice_amd import abi
    nodes = sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node")) \
        if os.path.isdir("/sys/devices/system/node") else []
    allowed = os.sched_getaffinity(0)
    seen = set()
    for node in nodes:
        cpus = abi.node_cpus(node)
        assert set(cpus) <= allowed
        assert not (set(cpus) & seen)
        seen |= set(cpus)
    if nodes:
        assert seen == allowed or seen <= allowed
    assert abi.node_cpus(-1) == [] and abi.node_cpus(100000) == []
    assert 1 <= abi.usable_cpus() <= len(allowed)


@pytest.mark.parametrize("cfg", [synth.C3, synth.C4, synth.FUZZ])
def test_group_split_plan_exact_when_small_balanced_when_large(cfg):
    """bt_group_split_plan (the split group calls use): identical to the exact split up to 4096
    tiles; above it, sampled, still tile-aligned, contiguous and within 2 % of balance."""
    from beatrice_amd import abi
    _, desc = synth.capture(cfg, 1 << 20, seed=7)
    ln = synth.desc_len(desc).astype(np.uint32)
    for model in (shard.group_cost(True, False, True), shard.group_cost(True, True, True, 16),
                  shard.group_cost(False, True, True, 8, 112)):
        for n in (1000, 4096 * 64, 4096 * 64 + 1, 700001, 1 << 20):
            for parts in (2, 3, 8):
                plan = abi.group_split(ln[:n], parts, model, plan=True)
                if (n + 63) // 64 <= 4096:
                    assert plan == shard.shard_bounds(ln[:n], parts, cost=model)
                    continue
                assert plan[0][0] == 0 and plan[-1][1] == n
                assert all(lo % 64 == 0 for lo, _ in plan) and all(plan[i][1] == plan[i + 1][0] for i in range(parts - 1))
                c = [int(shard.packet_cost(ln[lo:hi], model).sum()) for lo, hi in plan]
                assert max(c) / (sum(c) / parts) < 1.02, (n, parts, model, c)
