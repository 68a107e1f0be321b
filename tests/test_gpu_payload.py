"""GPU: PAYLOAD filters evaluated by the kernel (BT_K_PAYLOAD) — the
bit-parallel Shift-And form where the pattern is a union of linear class sequences, the byte
DFA otherwise — instead of being resumed on the host, checked against the compiled reference
(goldens; oracle/_ref on a live sample), the blobs' host executor (full size) and each other
(the same program compiled both ways, BT_OPT_PAYLOAD_DFA)."""
import ctypes

import numpy as np
import pytest

import oracle_lib as ol
from beatrice_amd import abi, synth
from conftest import load_golden
from golden_util import compare_decisions

pytestmark = pytest.mark.gpu

BUILTIN_HEADLINE = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
                    {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2}]


def _run(ctx, data, desc, records=False):
    run = abi.DeviceRun(ctx, data, desc, len(desc), records=records)
    run.run()
    out = run.fetch()
    run.free()
    return out


def test_payload_sets_decide_on_gpu(gpu_ctx):
    g, man = load_golden("http")
    n = len(g["desc"])
    gpu_decided = 0
    for s in man["captures"]["http"]["filter_sets"]:
        if not s.startswith("payload_"):
            continue
        filters = man["filter_sets"][s]
        prog = gpu_ctx.compile(filters)
        out = _run(gpu_ctx, g["data"], g["desc"])
        compare_decisions(out["decide"], g[f"code__{s}"], g[f"src__{s}"], filters, where=f"http/{s}")
        # every slot the DFA compiler took is decided on the device: no HOST code at it
        dslot = out["decide"] & 63
        host = (out["decide"] >> 6) == 3
        for k, slot in enumerate(prog):
            if abi.KINDS[slot.kind] == "PAYLOAD":
                assert not np.any(host & (dslot == k)), f"{s}: HOST decision at GPU slot {k}"
                gpu_decided += 1
    assert gpu_decided >= 20


@pytest.mark.parametrize("cfg", [synth.C3, synth.C4])
def test_payload_full_size_vs_host_executor(gpu_ctx, cfg):
    n = 1 << 20
    data, desc = synth.capture(cfg, n, seed=99)
    expr = "[\\x80-\\xff]{3}|\\d\\d"
    blob = abi.payload_dfa(expr)
    gpu_ctx.compile([{"type": abi.PAYLOAD, "expr": expr, "priority": 1}])
    assert abi.KINDS[gpu_ctx.program()[0].kind] == "PAYLOAD"
    out = _run(gpu_ctx, data, desc)
    off, ln = synth.desc_off(desc), synth.desc_len(desc)
    want = np.array([abi.payload_dfa_eval(blob, data[o:o + m]) for o, m in zip(off, ln)])
    got = (out["decide"] >> 6) == 0
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} differ, first {bad[:5]}"
    assert 0 < want.sum() < n


@pytest.mark.skipif(not ol.ref_available(), reason="oracle/_ref (compiled reference) not built")
def test_payload_chain_vs_reference_sample(gpu_ctx):
    """A chain with two GPU PAYLOAD slots between built-ins, against the reference's
    own PacketFilter (std::regex per packet) on a 64k-packet sample."""
    n = 1 << 16
    data, desc = synth.capture(synth.C3, n, seed=5)
    filters = BUILTIN_HEADLINE[:1] + [{"type": abi.PAYLOAD, "expr": "[\\x00-\\x1f][a-z]", "priority": 2},
                                      {"type": abi.PAYLOAD, "expr": "^..?\\d", "priority": 1},
                                      {"type": abi.PORT_RANGE, "expr": "0-40000", "priority": 0}]
    prog = gpu_ctx.compile(filters)
    assert [abi.KINDS[p.kind] for p in prog] == ["PROTO_EQ", "PAYLOAD", "PAYLOAD", "PORT"]
    out = _run(gpu_ctx, data, desc)
    code, src = ol.ref_filter(data, desc, n, filters)
    compare_decisions(out["decide"], code, src, filters, where="c3/payload_chain")
    assert not np.any((out["decide"] >> 6) == 3)


def test_payload_host_option_and_pool_limit():
    ctx = abi.Context(0, flags=abi.OPT_PAYLOAD_HOST)
    try:
        prog = ctx.compile([{"type": abi.PAYLOAD, "expr": "GET", "priority": 1}])
        assert abi.KINDS[prog[0].kind] == "HOST"
    finally:
        ctx.close()
    ctx = abi.Context(0)
    try:
        big = "GET|POST|PUT|HEAD|DELETE|OPTIONS|PATCH|CONNECT|TRACE"   # ~1 KB of tables each
        fs = [{"type": abi.PAYLOAD, "expr": big + "x" * k, "priority": -k} for k in range(40)]
        kinds = [abi.KINDS[p.kind] for p in ctx.compile(fs)]
        assert kinds[0] == "PAYLOAD" and "HOST" in kinds   # the 16 KiB pool fills, the rest stay on the host
        pool = ctypes.c_uint32(0)
        abi._check(abi.lib().bt_filter_dfa_pool(ctx.h, None, 0, ctypes.byref(pool)))
        assert 0 < pool.value <= 16384
    finally:
        ctx.close()


def test_host_batch_payload_past_staged_headers():
    """bt_parse_filter (host buffers, prefix staging): a GPU PAYLOAD slot reads
    applyPayloadFilter's window up to frame byte 174 (src/PacketFilter.cpp:293-309), past
    the 112-B header prefix staged for the walk. Frames longer than that with the match
    beyond byte 112 (IHL up to 15, so the window starts at byte 74) decide exactly as
    the compiled reference PacketFilter."""
    rng = np.random.default_rng(5)
    frames = []
    for i in range(3000):
        ihl = 5 + (i % 11)
        po = 14 + 4 * ihl
        ln = int(rng.integers(34, 260))
        f = bytearray(rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
        f[12:14] = b"\x08\x00"
        if ln > 14:
            f[14] = 0x40 | ihl
        at = po + int(rng.choice([0, 38, 60, 90, 95, 99]))   # the window holds bytes [po, po + 100)
        if i % 3 and at + 5 <= ln:
            f[at:at + 5] = b"MAGIC"
        frames.append(bytes(f))
    data, desc = synth.pack_frames(frames, align=1)
    n = len(desc)
    filters = [{"type": abi.PROTOCOL, "expr": "ip", "priority": 2},
               {"type": abi.PAYLOAD, "expr": "MAG+IC", "priority": 1}]
    ctx = abi.Context(0, host_chunk_packets=1000)
    try:
        prog = ctx.compile(filters)
        assert abi.KINDS[prog[1].kind] == "PAYLOAD"
        out = ctx.run_host(data, desc)
    finally:
        ctx.close()
    code, src = ol.ref_filter(data, desc, n, filters)
    assert not ((out["decide"] >> 6) == 3).any(), "the GPU DFA slot left packets to the host"
    compare_decisions(out["decide"], code, src, filters, where="host-batch payload")
    late = [i for i, f in enumerate(frames) if f.find(b"MAGIC") >= 112]
    assert len(late) > 100 and (code[late] == 0).sum() > 50


FORM_PATTERNS = ["GET|POST", "User-Agent: .*(bot|curl)", "^.{0,5}$", "\\s+$", "[\\x80-\\xff]{4,}", "passw(or)?d=",
                 "^\\x16\\x03[\\x00-\\x03]", "(?:GET|HEAD) /[^ ]* HTTP", "a.?b*c", "[0-9a-f]{2}[^a-z]?z+$"]


@pytest.mark.parametrize("cfg", [synth.C3, synth.FUZZ])
def test_bitpar_and_dfa_forms_agree(cfg):
    """Every FORM_PATTERNS regex takes the bit-parallel form by default (32- and 64-bit states,
    anchors, optional and repeated classes) and decides every packet of a 1M-packet capture
    exactly as the same slot compiled as a byte DFA; a 64k sample against the reference."""
    n = 1 << 20
    data, desc = synth.capture(cfg, n, seed=41)
    # plant some matches: payload bytes of every 7th frame rewritten with pattern-shaped text
    off, ln = synth.desc_off(desc), synth.desc_len(desc)
    words = [b"GET /", b"POST", b"User-Agent: x bot", b"passwd=", b"\x16\x03\x01", b"HEAD /a HTTP", b"abbbc"]
    for i in range(0, n, 7):
        o, m = int(off[i]), int(ln[i])
        if m > 60:
            w = words[(i // 7) % len(words)]
            at = o + 14 + 20 + (i % 13)
            if at + len(w) <= o + m:
                data[at:at + len(w)] = np.frombuffer(w, np.uint8)
    bp, dfa = abi.Context(0), abi.Context(0, flags=abi.OPT_PAYLOAD_DFA)
    try:
        for expr in FORM_PATTERNS:
            f = [{"type": abi.PAYLOAD, "expr": expr, "priority": 1}]
            assert abi.KINDS[bp.compile(f)[0].kind] == "PAYLOAD" and abi.KINDS[dfa.compile(f)[0].kind] == "PAYLOAD"
            blob = abi.payload_dfa(expr)
            assert blob[:2] == b"\xff\xff", f"/{expr}/ did not take the bit-parallel form"
            a, b = _run(bp, data, desc), _run(dfa, data, desc)
            bad = np.nonzero(a["decide"] != b["decide"])[0]
            assert len(bad) == 0, f"/{expr}/: {len(bad)} decisions differ between the forms, first {bad[:5]}"
            if ol.ref_available():
                k = 1 << 16
                code, src = ol.ref_filter(data, desc, k, f)
                compare_decisions(a["decide"][:k], code, src, f, where=f"{cfg}/bitpar /{expr}/")
    finally:
        dfa.close()
        bp.close()


@pytest.mark.parametrize("stride", [64, 128])
def test_fixed_stride_payload(gpu_ctx, stride):
    """Fixed-stride batches (no descriptors): 64-B frames use LDS rows of 17 dwords, not 33, so
    the window staging, its padding and the walks must stay inside them; matches planted at
    every offset of the window, frames with IP options and non-IPv4 frames, decided as the
    descriptor path and the compiled reference decide them."""
    rng = np.random.default_rng(stride)
    n = 64 * 300 + 17
    frames = []
    for i in range(n):
        f = bytearray(rng.integers(0, 256, stride, dtype=np.uint8).tobytes())
        f[12:14] = b"\x08\x00" if i % 11 else b"\x86\xdd"
        ihl = 5 + (i % 7 == 0) * (i % 5)
        f[14] = 0x40 | ihl
        po = 14 + 4 * ihl
        w = (b"GET", b"POST", b"GE", b"xPOSTx")[i % 4]
        at = po + (i * 7) % max(1, stride - po - len(w) + 1)
        if i % 3 and at + len(w) <= stride:
            f[at:at + len(w)] = w
        frames.append(bytes(f))
    data, desc = synth.pack_frames(frames, align=stride)
    assert np.all(synth.desc_off(desc) == np.arange(n) * stride)
    for expr in ("GET|POST", "ST$|^x?G", "[\\x80-\\xff]{3}|\\d\\d"):
        f = [{"type": abi.PAYLOAD, "expr": expr, "priority": 1}]
        assert abi.KINDS[gpu_ctx.compile(f)[0].kind] == "PAYLOAD"
        run = abi.DeviceRun(gpu_ctx, data[: n * stride], None, n, stride=stride, records=False)
        run.run()
        fixed = run.fetch()["decide"]
        run.free()
        by_desc = _run(gpu_ctx, data, desc)["decide"]
        bad = np.nonzero(fixed != by_desc)[0]
        assert len(bad) == 0, f"/{expr}/ stride {stride}: {len(bad)} fixed-stride decisions differ, first {bad[:5]}"
        blob = abi.payload_dfa(expr)
        want = np.array([abi.payload_dfa_eval(blob, data[i * stride:(i + 1) * stride]) for i in range(n)])
        got = (fixed >> 6) == 0
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, f"/{expr}/ stride {stride}: {len(bad)} differ from the host executor, first {bad[:5]}"
        assert 0 < want.sum() < n
        if ol.ref_available():
            code, src = ol.ref_filter(data, desc, n, f)
            compare_decisions(fixed, code, src, f, where=f"fixed{stride}/{expr}")
