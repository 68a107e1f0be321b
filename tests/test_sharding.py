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
