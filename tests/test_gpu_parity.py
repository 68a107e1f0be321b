"""GPU parity: the gfx950 path (through the C-ABI) against the golden fixtures from the
compiled reference and against the oracle on seeded captures. Bit-exact: records,
decision bytes, verdict words, compacted pass indices."""
import numpy as np
import pytest

import oracle_lib as ol
from beatrice_amd import abi, synth
from ring_util import umem_capture
from conftest import load_golden
from golden_util import CAPTURES, compare_decisions, eval_order

pytestmark = pytest.mark.gpu


def run_dev(ctx, data, desc, n, stride=0, records=True, filt=True):
    r = abi.DeviceRun(ctx, data, desc, n, stride=stride, records=records, decide=filt, verdict=filt,
                      pass_idx=filt)
    r.run()
    out = r.fetch()
    r.free()
    return out


def check_filter_outputs(out, n):
    dec = out["decide"]
    ver = out["verdict"]
    bits = np.unpackbits(ver.view(np.uint8), bitorder="little")[:n].astype(bool)
    assert np.array_equal(bits, (dec >> 6) == 0), "verdict bits != decide codes"
    tail = np.unpackbits(ver.view(np.uint8), bitorder="little")[n:]
    assert not tail.any(), "verdict bits set past n"
    exp_idx = np.nonzero(bits)[0]
    assert out["n_pass"] == len(exp_idx)
    assert np.array_equal(out["pass_idx"], exp_idx.astype(np.uint32)), "pass_idx not the ordered passing set"


@pytest.mark.parametrize("cap", CAPTURES)
def test_records_match_reference(gpu_ctx, cap):
    g, _ = load_golden(cap)
    n = len(g["desc"])
    gpu_ctx.compile([])
    out = run_dev(gpu_ctx, g["data"], g["desc"], n, records=True, filt=False)
    bad = np.nonzero((out["records"] != g["rec"]).any(axis=1))[0]
    assert len(bad) == 0, f"{cap}: {len(bad)} records differ; first {bad[:5]}"


@pytest.mark.parametrize("cap", CAPTURES)
def test_filters_match_reference(gpu_ctx, cap):
    g, man = load_golden(cap)
    n = len(g["desc"])
    for s in man["captures"][cap]["filter_sets"]:
        filters = man["filter_sets"][s]
        prog = gpu_ctx.compile(filters)
        assert [p.source_index for p in prog] == eval_order(filters)
        out = run_dev(gpu_ctx, g["data"], g["desc"], n, records=(s == "c3"), filt=True)
        compare_decisions(out["decide"], g[f"code__{s}"], g[f"src__{s}"], filters, where=f"{cap}/{s}")
        check_filter_outputs(out, n)
        if s == "c3":
            assert np.array_equal(out["records"], g["rec"])


@pytest.mark.parametrize("stride", [16, 32, 64, 128, 80, 200])
def test_fixed_stride_matches_oracle(gpu_ctx, stride):
    n = 70001
    data, desc = synth.capture(synth.C2, n)
    # re-pack the 64-B frames at `stride` (truncated or zero-padded to the stride)
    frames = data[:n * 64].reshape(n, 64)
    buf = np.zeros((n, stride), np.uint8)
    m = min(64, stride)
    buf[:, :m] = frames[:, :m]
    buf = buf.reshape(-1)
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
               {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
    gpu_ctx.compile(filters)
    out = run_dev(gpu_ctx, buf, None, n, stride=stride)
    rec, dec, npass = ol.oracle_run(buf, None, n, filters, stride=stride)
    assert np.array_equal(out["records"], rec)
    assert np.array_equal(out["decide"], dec)
    assert out["n_pass"] == npass
    check_filter_outputs(out, n)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 127, 128, 129, 191, 255, 256, 257, 69893, 70001, 70003, 1 << 17])
def test_fixed_stride_tile_groups_and_tails(gpu_ctx, n):
    """The 64-B parse+filter kernel (the headline's) may store a block's four tiles' decisions
    and verdict words at once: every tail form — a tile count not a multiple of 4, a group cut
    by n, n not a multiple of 4, a single tile — against the oracle, with and without the
    records."""
    data, desc = synth.capture(synth.C2, n, seed=0x7A11 + n)
    buf = np.ascontiguousarray(data[:n * 64])
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
               {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
    gpu_ctx.compile(filters)
    rec, dec, npass = ol.oracle_run(buf, None, n, filters, stride=64)
    for records in (True, False):
        out = run_dev(gpu_ctx, buf, None, n, stride=64, records=records)
        if records:
            assert np.array_equal(out["records"], rec)
        assert np.array_equal(out["decide"], dec)
        assert out["n_pass"] == npass
        check_filter_outputs(out, n)


@pytest.mark.parametrize("cfg,n", [(synth.C3, 1 << 20), (synth.C4, 1 << 20), (synth.FUZZ, 1 << 20),
                                   (synth.FUZZ, 777)])
def test_seeded_captures_match_oracle(gpu_ctx, cfg, n):
    data, desc = synth.capture(cfg, n, seed=0xC0FFEE + cfg)
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
               {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1},
               {"type": abi.BPF, "expr": "udp tcp", "priority": 0}]
    gpu_ctx.compile(filters)
    out = run_dev(gpu_ctx, data, desc, n)
    rec, dec, npass = ol.oracle_run(data, desc, n, filters)
    bad = np.nonzero((out["records"] != rec).any(axis=1))[0]
    assert len(bad) == 0, f"{len(bad)} records differ; first {bad[:5]}"
    assert np.array_equal(out["decide"], dec)
    assert out["n_pass"] == npass
    check_filter_outputs(out, n)


@pytest.mark.parametrize("cap,layout", [("c3", "tiled"), ("c4", "tiled"), ("fuzz", "tiled"), ("edge", "tiled"),
                                        ("c4", "planes"), ("edge", "aos")])
def test_host_batch_path(cap, layout):
    """bt_parse_filter: host buffers, prefix gather into pinned staging, multi-chunk
    double-buffered pipeline (chunk 1024 packets). The pipeline copies bt_rec AoS back
    whatever record layout the context's flags select for device batches."""
    g, man = load_golden(cap)
    n = len(g["desc"])
    flags = {"tiled": 0, "planes": abi.OPT_RECORDS_PLANES, "aos": abi.OPT_RECORDS_AOS}[layout]
    ctx = abi.Context(0, host_chunk_packets=1000, flags=flags)
    try:
        filters = man["filter_sets"]["c3"]
        ctx.compile(filters)
        out = ctx.run_host(g["data"], g["desc"])
        assert np.array_equal(out["records"], g["rec"])
        compare_decisions(out["decide"], g["code__c3"], g["src__c3"], filters, where=cap)
        bits = np.unpackbits(out["verdict"].view(np.uint8), bitorder="little")[:n].astype(bool)
        assert np.array_equal(np.nonzero(bits)[0].astype(np.uint32), out["pass_idx"])
    finally:
        ctx.close()


@pytest.mark.parametrize("cfg", [synth.C2, synth.C3])
def test_full_size_batch_properties(gpu_ctx, cfg):
    """BASELINE size (16M packets): size-independent checks — a 64Ki-packet random
    sample against the oracle, verdict/decide/pass_idx consistency, monotone indices."""
    n = 1 << 24
    data, desc = synth.capture(cfg, n)
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
               {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
    gpu_ctx.compile(filters)
    stride = 64 if cfg == synth.C2 else 0
    out = run_dev(gpu_ctx, data, None if stride else desc, n, stride=stride)
    check_filter_outputs(out, n)
    rng = np.random.default_rng(7)
    idx = np.sort(rng.choice(n, 65536, replace=False))
    sub_desc = desc[idx]
    rec, dec, _ = ol.oracle_run(data, sub_desc, len(idx), filters)
    assert np.array_equal(out["records"][idx], rec)
    assert np.array_equal(out["decide"][idx], dec)
    assert np.all(np.diff(out["pass_idx"].astype(np.int64)) > 0)


def test_full_size_c4_streamed(gpu_ctx):
    """C4 (QinQ / IPv6 / IHL + TCP options, frames at 2-mod-4 offsets) at the size bench.py
    times it: 16,777,216 packets, a multi-GB capture generated range by range and streamed
    into HBM the way bench.py's Capture does, so the host never holds it whole. Checked: a
    64Ki-packet random sample plus the first and last tiles against the oracle (records and
    decisions), and the verdict / decision / pass-list properties over all 16M."""
    n = 1 << 24
    cfg, seed = synth.C4, synth.SEEDS[synth.C4]
    desc, nbytes = synth.layout(cfg, n, seed)
    off, ln = synth.desc_off(desc), synth.desc_len(desc)
    assert (off % 4 == 2).mean() > 0.99   # the 2-mod-4 frame starts the bench times
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
               {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
    gpu_ctx.compile(filters)
    rng = np.random.default_rng(0xC4)
    idx = np.unique(np.concatenate([rng.choice(n, 65536, replace=False), np.arange(64),
                                    np.arange(n - 64, n)]))
    run = abi.DeviceRun(gpu_ctx, None, desc, n, data_bytes=nbytes + synth.FILL_PAD)
    try:
        frames = []   # the sampled frames, copied out of each streamed range
        chunk = 1 << 20
        for i in range(0, n, chunk):
            j = min(n, i + chunk)
            buf, b0, nb = synth.fill_range(cfg, seed, desc, i, j)
            run.upload_data(buf[:nb], b0)
            for k in idx[(idx >= i) & (idx < j)]:
                s = int(off[k]) - b0
                frames.append(buf[s:s + int(ln[k])].copy())
            del buf
        run.run()
        out = run.fetch()
    finally:
        run.free()
    check_filter_outputs(out, n)
    assert np.all(np.diff(out["pass_idx"].astype(np.int64)) > 0)
    # the sample packed at the frames' own 4-byte phase (alignment changes nothing on the CPU)
    data, sdesc = synth.pack_frames(frames, align=4, shift=2)
    rec, dec, _ = ol.oracle_run(data, sdesc, len(idx), filters)
    bad = np.nonzero((out["records"][idx] != rec).any(axis=1))[0]
    assert len(bad) == 0, f"{len(bad)} sampled C4 records differ; first packets {idx[bad[:5]]}"
    assert np.array_equal(out["decide"][idx], dec)


def test_edge_batches(gpu_ctx):
    gpu_ctx.compile([{"type": abi.PROTOCOL, "expr": "udp"}])
    # n = 0
    data = np.zeros(256, np.uint8)
    out = run_dev(gpu_ctx, data, np.zeros(0, np.uint64), 0)
    assert out["n_pass"] == 0
    # n = 1, zero-length frame; a 65535-byte frame; a descriptor past the buffer end
    big = np.zeros(70000, np.uint8)
    big[12:14] = [0x08, 0x00]
    big[14] = 0x45
    big[23] = 17
    desc = synth.make_desc([0, 0, 60000], [0, 65535, 9000])
    out = run_dev(gpu_ctx, big, desc[:1], 1)
    assert out["records"][0, 24] == abi.L_ETH and out["records"][0, 25] == 0
    rec, dec, _ = ol.oracle_run(big, desc[:2], 2, [{"type": abi.PROTOCOL, "expr": "udp"}])
    out = run_dev(gpu_ctx, big, desc[:2], 2)
    assert np.array_equal(out["records"], rec) and np.array_equal(out["decide"], dec)
    out = run_dev(gpu_ctx, big, desc, 3)   # third frame runs past `bytes`: no fault
    assert out["records"].shape == (3, 96)


def test_too_many_filters(gpu_ctx):
    fs = [{"type": abi.BPF, "expr": "udp", "priority": i} for i in range(65)]
    with pytest.raises(abi.BtError):
        gpu_ctx.compile(fs)
    prog = gpu_ctx.compile(fs[:64])
    assert len(prog) == 64 and prog[0].source_index == 63


def test_graph_replay_outputs(gpu_ctx):
    """BT_OPT_GRAPH: the timed steps replayed as one hipGraph produce the same outputs."""
    n = 200003
    data, desc = synth.capture(synth.C3, n, seed=99)
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
    ctx = abi.Context(0, flags=abi.OPT_GRAPH)
    try:
        ctx.compile(filters)
        r = abi.DeviceRun(ctx, data, desc, n)
        span, main = ctx.time_device(r.batch, r.outs, 3)    # builds the graph
        span2, main2 = ctx.time_device(r.batch, r.outs, 3)  # replays it
        assert main == -1.0 and main2 == -1.0 and span2 > 0
        out = r.fetch()
        r.free()
    finally:
        ctx.close()
    rec, dec, npass = ol.oracle_run(data, desc, n, filters)
    assert np.array_equal(out["records"], rec) and np.array_equal(out["decide"], dec)
    check_filter_outputs(out, n)


def test_zero_copy_umem_ingest(gpu_ctx):
    """AF_XDP UMEM + RX xdp_desc ring consumed zero-copy — both
    registered with bt_host_register, the kernel reads the header windows over PCIe."""
    n = 50000
    data, desc = synth.capture(synth.C3, n, seed=31)
    mm, umem, xdp, packed = umem_capture(data, desc)
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
               {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
    gpu_ctx.compile(filters)
    xdp = abi.host_copy(xdp)   # the RX ring on pages of its own, as the kernel maps it
    d_umem = gpu_ctx.register(umem)
    d_xdp = gpu_ctx.register(xdp)
    try:
        r = abi.DeviceRun(gpu_ctx, np.zeros(256, np.uint8), None, n, stride=1)
        r.batch = abi.Batch(d_umem, d_xdp, 0, n, umem.nbytes, abi.DESC_XDP, 0)
        r.run()
        out = r.fetch()
        r.free()
    finally:
        gpu_ctx.unregister(xdp)
        gpu_ctx.unregister(umem)
    rec, dec, npass = ol.oracle_run(umem, packed, n, filters)
    assert np.array_equal(out["records"], rec)
    assert np.array_equal(out["decide"], dec)
    check_filter_outputs(out, n)
    del umem
    mm.close()


def test_zero_copy_outputs(gpu_ctx):
    """Outputs written by the kernel straight into registered host memory."""
    n = 30000
    data, desc = synth.capture(synth.C4, n, seed=77)
    filters = [{"type": abi.BPF, "expr": "tcp", "priority": 1}]
    gpu_ctx.compile(filters)
    # every registered buffer on pages of its own (registration is in whole pages)
    data, desc = abi.host_copy(data), abi.host_copy(desc)
    h_rec = abi.host_array(((n + 63) // 64) * 6144)
    h_dec = abi.host_array(n)
    h_ver = abi.host_array((n + 63) // 64, np.uint64)
    d_data, d_desc = gpu_ctx.register(data), gpu_ctx.register(desc)
    aliases = [gpu_ctx.register(x) for x in (h_rec, h_dec, h_ver)]
    try:
        batch = abi.Batch(d_data, d_desc, 0, n, data.nbytes, abi.DESC_PACKED, 0)
        gpu_ctx.run_device(batch, abi.Outputs(aliases[0], n, aliases[2], aliases[1], None, None))
        gpu_ctx.synchronize()
    finally:
        for x in (h_rec, h_dec, h_ver, data, desc):
            gpu_ctx.unregister(x)
    rec, dec, _ = ol.oracle_run(data, desc, n, filters)
    assert np.array_equal(abi.untile_records(h_rec, n), rec)
    assert np.array_equal(h_dec, dec)
    bits = np.unpackbits(h_ver.view(np.uint8), bitorder="little")[:n].astype(bool)
    assert np.array_equal(bits, (dec >> 6) == 0)


@pytest.mark.parametrize("layout", ["tiled", "planes", "aos"])
@pytest.mark.parametrize("cap", ["c4", "fuzz", "edge"])
def test_record_layouts(cap, layout):
    """Every device record layout (packed tiled, packed plane-major, bt_rec AoS) rebuilds
    the reference's records, with and without a filter program."""
    flags = {"tiled": 0, "planes": abi.OPT_RECORDS_PLANES, "aos": abi.OPT_RECORDS_AOS}[layout]
    g, man = load_golden(cap)
    n = len(g["desc"])
    ctx = abi.Context(0, flags=flags)
    try:
        for filters in ([], man["filter_sets"]["c3"]):
            ctx.compile(filters)
            out = run_dev(ctx, g["data"], g["desc"], n, records=True, filt=bool(filters))
            bad = np.nonzero((out["records"] != g["rec"]).any(axis=1))[0]
            assert len(bad) == 0, f"{cap}/{layout}: {len(bad)} records differ; first {bad[:5]}"
            if filters:
                compare_decisions(out["decide"], g["code__c3"], g["src__c3"], filters, where=f"{cap}/{layout}")
    finally:
        ctx.close()


# Every form of the main kernel launch_main can pick, on one ragged capture: the
# counted-wait pipeline (default in descriptor mode; a deep per-wave loop with 4 waves;
# blocked tile order; forced wide / two-round loads) and bt_parse_filter_main (no
# prefetch; default cache policy). Parse+filter, parse-only and filter-only, at batch
# sizes 1, 63, 65 and 20,037 (not a multiple of the 64-packet tile).
KERNEL_FORMS = {
    "pipe": dict(flags=0),
    "pipe_4_waves": dict(flags=0, grid_waves=4),
    "pipe_blocked": dict(flags=abi.OPT_TILE_BLOCKED, grid_waves=64),
    "pipe_wide_always": dict(flags=abi.OPT_WIDE_ALWAYS),
    "pipe_wide_never": dict(flags=abi.OPT_WIDE_NEVER),
    "main_no_prefetch": dict(flags=abi.OPT_NO_PREFETCH),
    "main_cache_default": dict(flags=abi.OPT_CACHE_DEFAULT, grid_waves=8),
}


@pytest.mark.parametrize("form", list(KERNEL_FORMS))
def test_kernel_forms_agree(form):
    data, desc = synth.capture(synth.FUZZ, 20037, seed=11)
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
               {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
    ctx = abi.Context(0, **KERNEL_FORMS[form])
    try:
        ctx.compile(filters)
        for n in (1, 63, 65, len(desc)):
            d = np.ascontiguousarray(desc[:n])
            rec, dec, npass = ol.oracle_run(data, d, n, filters)
            out = run_dev(ctx, data, d, n)
            assert np.array_equal(out["records"], rec), f"{form} n={n}: records"
            assert np.array_equal(out["decide"], dec), f"{form} n={n}: decisions"
            assert out["n_pass"] == npass
            check_filter_outputs(out, n)
            out = run_dev(ctx, data, d, n, filt=False)
            assert np.array_equal(out["records"], rec), f"{form} n={n}: parse-only records"
            out = run_dev(ctx, data, d, n, records=False)
            assert np.array_equal(out["decide"], dec), f"{form} n={n}: filter-only decisions"
            check_filter_outputs(out, n)
    finally:
        ctx.close()


FAR = 3 << 29   # 1.5 GiB


@pytest.mark.parametrize("cfg", [synth.FUZZ, synth.C4])
@pytest.mark.parametrize("which", ["odd_far", "even_far", "half_tiles_far"])
def test_far_descriptors(gpu_ctx, cfg, which):
    """Descriptors of one tile spread over 1.5 GiB: the capture is stored twice, 1.5 GiB
    apart, and some packets' descriptors point into the far
    copy (every other packet, or every other half tile). The 64-bit window addressing of
    round A / round B must give the oracle's results on the original capture. (A 32-bit
    form — offsets from a per-tile base, far windows deferred to round B — passed this
    test but measured no faster: C3 0.505 vs 0.505 ms, C4 0.948 vs 0.944 ms; that form
    needs a range of 1 GiB around a tile's lane 0.)"""
    n = 20037
    data, desc = synth.capture(cfg, n, seed=0xFA2 + cfg)
    off, ln = synth.desc_off(desc), synth.desc_len(desc)
    i = np.arange(n)
    move = {"odd_far": i % 2 == 1, "even_far": i % 2 == 0, "half_tiles_far": (i // 32) % 2 == 1}[which]
    d2 = synth.make_desc(off + np.where(move, FAR, 0), ln)
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
               {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
    gpu_ctx.compile(filters)
    rec, dec, npass = ol.oracle_run(data, desc, n, filters)
    r = abi.DeviceRun(gpu_ctx, None, d2, n, data_bytes=FAR + data.nbytes)
    try:
        r.upload_data(data, 0)
        r.upload_data(data, FAR)
        r.run()
        out = r.fetch()
    finally:
        r.free()
    bad = np.nonzero((out["records"] != rec).any(axis=1))[0]
    assert len(bad) == 0, f"{len(bad)} records differ; first {bad[:5]}"
    assert np.array_equal(out["decide"], dec)
    assert out["n_pass"] == npass
    check_filter_outputs(out, n)


def test_repeated_runs_are_identical(gpu_ctx):
    """The same 1M-packet C4 batch through the main kernel 16 times: records, decisions and
    pass lists never change (a wait that retired too early — the counted vmcnt waits of
    bt_parse_filter_pipe — would show up as run-to-run differences), and match the oracle."""
    n = 1 << 20
    data, desc = synth.capture(synth.C4, n, seed=0xBEEF)
    filters = [{"type": abi.PROTOCOL, "expr": "tcp", "priority": 2},
               {"type": abi.PORT_RANGE, "expr": "1-40000", "priority": 1}]
    gpu_ctx.compile(filters)
    r = abi.DeviceRun(gpu_ctx, data, desc, n)
    try:
        r.run()
        first = r.fetch()
        rec, dec, npass = ol.oracle_run(data, desc, n, filters)
        assert np.array_equal(first["records"], rec) and np.array_equal(first["decide"], dec)
        assert first["n_pass"] == npass
        for _ in range(15):
            r.run()
            out = r.fetch()
            for k in ("records", "decide", "verdict", "pass_idx"):
                assert np.array_equal(out[k], first[k]), k
            assert out["n_pass"] == first["n_pass"]
    finally:
        r.free()


@pytest.mark.parametrize("fset", ["c3", "mixed", "throw_after", "empty"])
def test_fixed_stride_headline_kernel_on_reference_fixture(fset):
    """The headline's kernel form — fixed 64-B stride, no descriptors
    (bt_parse_filter_main<2, tiled, filter>) — on the c1 golden frames (10k x 64 B at
    stride 64) against the compiled reference's own records and applyFilters outcomes,
    not only against the C restatement."""
    g, man = load_golden("c1")
    n = len(g["desc"])
    assert (synth.desc_off(g["desc"]) == np.arange(n) * 64).all() and (synth.desc_len(g["desc"]) == 64).all()
    filters = man["filter_sets"][fset]
    ctx = abi.Context(0)
    try:
        ctx.compile(filters)
        out = run_dev(ctx, g["data"], None, n, stride=64)
        assert np.array_equal(out["records"], g["rec"]), "records differ from the reference fixture"
        host = compare_decisions(out["decide"], g[f"code__{fset}"], g[f"src__{fset}"], filters, where=f"c1/{fset}")
        assert len(host) == 0
        check_filter_outputs(out, n)
        out = run_dev(ctx, g["data"], None, n, stride=64, filt=False)   # the C2 parse-only form
        assert np.array_equal(out["records"], g["rec"])
    finally:
        ctx.close()


@pytest.mark.parametrize("cfg", [synth.FUZZ, synth.C3])
def test_random_programs_match_oracle(gpu_ctx, cfg):
    """40 seeded random programs over the built-in kinds (tests/random_programs.py: the
    reference's expression quirks, throwing expressions, disabled filters): decision
    bytes, verdict words and pass lists equal the oracle's, which
    tests/test_random_programs.py pins against the compiled reference."""
    from random_programs import random_programs
    n = 20037
    data, desc = synth.capture(cfg, n, seed=0x5B + cfg)
    for i, prog in enumerate(random_programs(0xF117E3 + cfg, 40)):
        gpu_ctx.compile(prog)
        out = run_dev(gpu_ctx, data, desc, n, records=False)
        _, dec, npass = ol.oracle_run(data, desc, n, prog, parse=False)
        bad = np.nonzero(out["decide"] != dec)[0]
        assert len(bad) == 0, f"program {i} {prog}: {len(bad)} decisions differ, first {bad[:5]}"
        assert out["n_pass"] == npass, f"program {i}"
        check_filter_outputs(out, n)


def test_async_pipeline_batches_match_oracle():
    """bt_parse_filter_device_async over a stream of 6 different batches (C3 and fixed-stride
    C2, alternating two output sets as the API asks): each compaction runs on the context's
    compaction stream beside the next batch's main kernel, with the double-buffered
    workspace alternating under it. Every batch's records, decisions, verdicts and ordered
    pass list equal the oracle's."""
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
               {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
    ctx = abi.Context(0)
    runs, caps = [], []
    try:
        ctx.compile(filters)
        for i in range(6):
            n = 50000 + 4099 * i
            if i % 2:
                data, desc = synth.capture(synth.C3, n, seed=0xA5 + i)
                caps.append((data, desc, n, 0))
                runs.append(abi.DeviceRun(ctx, data, desc, n))
            else:
                data, desc = synth.capture(synth.C2, n, seed=0xA5 + i)
                caps.append((data, None, n, 64))
                runs.append(abi.DeviceRun(ctx, data, None, n, stride=64))
        for rnd in range(2):   # two rounds: batch i's outputs rewritten by the second round
            for r in runs:
                ctx.run_device_async(r.batch, r.outs)
        ctx.synchronize()
        for (data, desc, n, stride), r in zip(caps, runs):
            out = r.fetch()
            rec, dec, npass = ol.oracle_run(data, desc, n, filters, stride=stride)
            assert np.array_equal(out["records"], rec)
            assert np.array_equal(out["decide"], dec)
            assert out["n_pass"] == npass
            check_filter_outputs(out, n)
    finally:
        for r in runs:
            r.free()
        ctx.close()


def test_pipelined_timing_outputs():
    """BT_OPT_PIPELINE (bench's pipelined steps): after a timed run of 8 steps the outputs
    are those of one synchronous call."""
    n = 1 << 20
    data, desc = synth.capture(synth.C3, n, seed=0x77)
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2}]
    ctx = abi.Context(0, flags=abi.OPT_PIPELINE)
    try:
        ctx.compile(filters)
        r = abi.DeviceRun(ctx, data, desc, n)
        t = ctx.time_device_ex(r.batch, r.outs, 8)
        assert t.span_ms > 0 and t.main_ms > 0
        out = r.fetch()
        rec, dec, npass = ol.oracle_run(data, desc, n, filters)
        assert np.array_equal(out["records"], rec) and np.array_equal(out["decide"], dec)
        assert out["n_pass"] == npass
        check_filter_outputs(out, n)
        r.free()
    finally:
        ctx.close()


def test_staged_host_copies_round_trip(gpu_ctx):
    """bt_memcpy_h2d / bt_memcpy_d2h go through the context's two pinned 8-MiB chunks:
    sizes around and across the chunk boundary, from and into unaligned host views,
    round-trip bit-exactly (and a device-side fill proves the bytes really crossed)."""
    rng = np.random.default_rng(5)
    chunk = 8 << 20
    for size in (1, 15, 4096 + 3, chunk - 1, chunk, chunk + 17, 3 * chunk + 5):
        src = rng.integers(0, 256, size=size + 3, dtype=np.uint8)[3:]      # unaligned view
        buf = gpu_ctx.alloc(size + 64)
        buf.zero()
        buf.upload(src)
        back = np.zeros(size + 1, np.uint8)[1:]                             # unaligned view
        buf.download(back)
        assert np.array_equal(back, src), size
        buf.zero()
        buf.download(back)
        assert not back.any(), size
        buf.free()


@pytest.mark.parametrize("layout", ["tiled", "planes", "aos", "filter_only"])
def test_fixed_stride_layouts_long_program(layout):
    """The fixed-stride kernel in every output form (its late-issue variant serves tiled,
    plane-major and filter-only, AoS keeps the plain order) with a 6-slot program, so slots
    0-3 run from registers side by side and slots 4-5 from the slot-by-slot loop, each
    deciding for some packets; bit-exact against the oracle."""
    n = 20037
    data, _ = synth.capture(synth.C2, n, seed=0x51D)
    filters = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 9},
               {"type": abi.BPF, "expr": "udp tcp", "priority": 8},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 7},
               {"type": abi.PORT_RANGE, "expr": "0-65535", "priority": 6},
               {"type": abi.IP_RANGE, "expr": "10.0.0.0/9", "priority": 5},
               {"type": abi.PORT_RANGE, "expr": "1000-30000", "priority": 4}]
    flags = {"tiled": 0, "planes": abi.OPT_RECORDS_PLANES, "aos": abi.OPT_RECORDS_AOS, "filter_only": 0}[layout]
    ctx = abi.Context(0, flags=flags)
    try:
        ctx.compile(filters)
        out = run_dev(ctx, data, None, n, stride=64, records=layout != "filter_only")
    finally:
        ctx.close()
    rec, dec, npass = ol.oracle_run(data, None, n, filters, stride=64)
    slots = dec & 0x3F
    assert (slots[(dec >> 6) == 1] >= 4).any(), "no packet decided by a slot past the hot ones"
    if layout != "filter_only":
        assert np.array_equal(out["records"], rec)
    assert np.array_equal(out["decide"], dec)
    assert out["n_pass"] == npass
    check_filter_outputs(out, n)
