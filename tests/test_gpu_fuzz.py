"""GPU: a time-bounded randomized parity sweep over every entry form.

Each round draws a capture (C2 / C3 / C4 / fuzz frames, a random seed and a packet count
that is rarely a tile multiple), a random program over the built-in kinds (the reference's
expression quirks, throwing expressions, disabled filters; tests/random_programs.py) and one
entry form of the product:
  host      bt_parse_filter: frames in host memory, the host pipeline (records sometimes)
  ptrs      bt_parse_filter_ptrs: one pointer per frame (the std::vector<Packet> form)
  device    bt_parse_filter_device: batch resident in device memory
  mapped    bt_group_parse_filter_mapped over 1-3 shared-device members: frames and outputs
            in registered host memory, read in place over PCIe (the lean first round)
  grouphost bt_group_parse_filter over 2-3 members (split or routed)
and checks decisions (and records when asked, and the verdict words / pass list) against the
oracle (tests/oracle_lib.py, pinned by the compiled reference's goldens). The sweep runs for
BT_FUZZ_SECONDS (default 15 s in the suite; a longer run is the same test with a larger
value) and prints one line per round.
"""
import os
import time

import numpy as np
import pytest

import oracle_lib as ol
from beatrice_amd import abi, synth
from random_programs import random_programs

pytestmark = pytest.mark.gpu

FORMS = ("host", "ptrs", "device", "mapped", "grouphost")


def _seed():
    """The sweep's seed: fixed in the suite (a failure reproduces), BT_FUZZ_SEED=random for a
    fresh one, or a given number."""
    e = os.environ.get("BT_FUZZ_SEED", "0xB1A5")
    return int(time.time()) & 0xFFFFFF if e == "random" else int(e, 0)


def _check(out, dec, n, npass, where):
    bad = np.nonzero(out["decide"][:n] != dec)[0]
    assert len(bad) == 0, f"{where}: {len(bad)} decisions differ, first {bad[:5]}; evidence {out.get('evidence')}"
    if out.get("verdict") is not None:
        bits = np.unpackbits(out["verdict"].view(np.uint8), bitorder="little")[:n].astype(bool)
        assert np.array_equal(bits, (dec >> 6) == 0), f"{where}: verdict words"
    if out.get("pass_idx") is not None:
        exp = np.nonzero((dec >> 6) == 0)[0].astype(np.uint32)
        assert out["n_pass"] == npass == len(exp) and np.array_equal(out["pass_idx"], exp), f"{where}: pass list"


class Arena:
    """A group's registered host buffers, registered once for the whole sweep (as a
    deployment registers its UMEM or ring once) and refilled every round: the capture is copied
    in, the outputs are poisoned (0xFF) so that a byte the device did not write shows up. Only
    with BT_FUZZ_ARENA=1; the default registers every round's own buffers (below)."""
    DATA = 128 << 20
    N = 70000

    def __init__(self, grp):
        self.grp = grp
        tiles = (self.N + 63) // 64
        self.data = abi.host_array(self.DATA)
        self.desc = abi.host_array(self.N, np.uint64)
        self.rec = abi.host_array(tiles * 6144)
        self.dec = abi.host_array(tiles * 64)
        self.ver = abi.host_array(tiles, np.uint64)
        self.held = [self.data, self.desc, self.rec, self.dec, self.ver]
        for a in self.held:
            grp.register(a)

    def close(self):
        for a in self.held:
            self.grp.unregister(a)


def _ranges(mask):
    idx = np.nonzero(mask)[0]
    if not len(idx):
        return []
    cuts = np.nonzero(np.diff(idx) > 1)[0]
    return [(int(s), int(e) + 1) for s, e in zip(np.concatenate([[idx[0]], idx[cuts + 1]]),
                                               np.concatenate([idx[cuts], [idx[-1]]]))][:8]


def _evidence(ctx, grp, batch, outs, data, desc, h_dec, h_ver, expect, n):
    """A mapped round whose decisions differ, examined while its buffers are still registered:
    the same call again, and the device's own copy (extract kernel, through the alias the mapped
    kernels read) of the capture and of its descriptors, compared with the host bytes."""
    import ctypes
    ev = {"first_bad": np.nonzero(h_dec[:n] != expect)[0][:12].tolist(),
          "got": h_dec[np.nonzero(h_dec[:n] != expect)[0][:12]].tolist()}
    h_dec.fill(0xFF)
    h_ver.fill(0xFFFFFFFFFFFFFFFF)
    grp.run_mapped(batch, outs)
    ev["rerun_bad"] = int(np.count_nonzero(h_dec[:n] != expect))
    for name, arr in (("data", data), ("desc", desc.view(np.uint8))):
        nb = arr.nbytes // 256 * 256
        if not nb:
            continue
        al = ctypes.c_void_p(0)
        if abi.lib().bt_host_alias(arr.ctypes.data, nb, 0, ctypes.byref(al)) != 0:
            ev[name] = "no alias"
            continue
        ex = abi.DeviceExtract(ctx, None, None, nb // 256, [(0, 256, abi.FT_BYTES, 0)],
                               batch=abi.Batch(al.value, None, 256, nb // 256, nb, 0, 0))
        ex.run()
        img = ex.fetch()[2].reshape(-1)
        ex.free()
        diff = img[:nb] != arr[:nb]
        ev[name] = {"host": hex(arr.ctypes.data), "alias": hex(al.value), "bytes_differ": int(diff.sum()),
                    "ranges": _ranges(diff), "device_zero_frac": float((img[:nb][diff] == 0).mean()) if diff.any() else None}
    return ev


def _mapped(grp, data, desc, n, records, arena=None, expect=None, ctx=None):
    """One mapped round. By default every buffer is the round's own: the capture and its
    descriptors copied to fresh pages, fresh output pages poisoned with 0xFF, all registered
    before the call and unregistered after it — thousands of registrations come and go at
    recycled addresses over a sweep, the form round 5's one difference showed up in
    (DESIGN.md §5). Registration is in whole pages, so each buffer has pages of its own
    (abi.host_array)."""
    tiles = max(1, (n + 63) // 64)
    pidx = np.zeros(max(n, 1), np.uint32)
    npass = np.zeros(1, np.uint32)
    if arena is not None and data.nbytes <= Arena.DATA and n <= Arena.N:
        arena.data[:data.nbytes] = data
        arena.desc[:n] = desc[:n]
        data, desc = arena.data[:data.nbytes], arena.desc
        h_rec = arena.rec[:tiles * 6144] if records else None
        h_dec, h_ver = arena.dec[:tiles * 64], arena.ver[:tiles]
        held = []
    else:
        data, desc = abi.host_copy(data), abi.host_copy(desc)
        h_rec = abi.host_array(tiles * 6144) if records else None
        h_dec = abi.host_array(tiles * 64)
        h_ver = abi.host_array(tiles, np.uint64)
        held = [a for a in (data, desc, h_rec, h_dec, h_ver) if a is not None]
    h_dec.fill(0xFF)
    h_ver.fill(0xFFFFFFFFFFFFFFFF)
    for a in held:
        grp.register(a)
    batch = abi.Batch(data.ctypes.data, desc.ctypes.data, 0, n, data.nbytes, abi.DESC_PACKED, 0)
    outs = abi.Outputs(None if h_rec is None else h_rec.ctypes.data, n, h_ver.ctypes.data,
                       h_dec.ctypes.data, pidx.ctypes.data, npass.ctypes.data)
    evidence = None
    try:
        grp.run_mapped(batch, outs)
        out = {"decide": h_dec[:n].copy(), "verdict": h_ver.copy(), "pass_idx": pidx[:int(npass[0])].copy(),
               "n_pass": int(npass[0]), "records": abi.untile_records(h_rec, n) if records else None}
        if expect is not None and ctx is not None and not np.array_equal(out["decide"], expect):
            evidence = _evidence(ctx, grp, batch, outs, data, desc, h_dec, h_ver, expect, n)
    finally:
        for a in held:
            grp.unregister(a)
    out["evidence"] = evidence
    return out


def _arena(arenas, key, grp):
    if os.environ.get("BT_FUZZ_ARENA", "0") in ("", "0"):
        return None
    if key not in arenas:
        arenas[key] = Arena(grp)
    return arenas[key]


def test_randomized_parity_sweep():
    seconds = float(os.environ.get("BT_FUZZ_SECONDS", "15"))
    seed0 = _seed()
    rng = np.random.default_rng(seed0)
    print(f"fuzz seed {seed0:#x}, {seconds:.0f} s", flush=True)
    ctx = abi.Context(0)
    groups = {}
    arenas = {}
    t_end = time.time() + seconds
    rounds = 0
    try:
        while time.time() < t_end or rounds < len(FORMS):
            cfg = [synth.C2, synth.C3, synth.C4, synth.FUZZ][int(rng.integers(0, 4))]
            n = int(rng.choice([1, 63, 64, 65, 127, 4097, int(rng.integers(1, 70000))]))
            cap_seed = int(rng.integers(1, 1 << 30))
            data, desc = synth.capture(cfg, n, seed=cap_seed)
            if data.nbytes < 64:   # fuzz frames of length 0: a registrable buffer all the same
                data = np.concatenate([data, np.zeros(64, np.uint8)])
            prog = random_programs(int(rng.integers(1, 1 << 30)), 1)[0]
            if rng.random() < 0.2:   # the metric's own set
                prog = [{"type": abi.PROTOCOL, "expr": "udp", "priority": 3},
                        {"type": abi.IP_RANGE, "expr": "10.0.0.0/8", "priority": 2},
                        {"type": abi.PORT_RANGE, "expr": "1000-2000", "priority": 1}]
            form = FORMS[rounds % len(FORMS)] if rounds < len(FORMS) else FORMS[int(rng.integers(0, len(FORMS)))]
            records = bool(rng.random() < 0.4)
            where = f"round {rounds} form {form} cfg {cfg} n {n} seed {cap_seed:#x} records {records} program {prog}"
            rec, dec, npass = ol.oracle_run(data, desc, n, prog, parse=records)
            if form in ("host", "ptrs", "device"):
                ctx.compile(prog)
                if form == "host":
                    out = ctx.run_host(data, desc, records=records)
                elif form == "ptrs":
                    off, ln = synth.desc_off(desc), synth.desc_len(desc)
                    frames = [data[int(o):int(o) + int(l)].tobytes() for o, l in zip(off, ln)]
                    grp = groups.setdefault(1, abi.Group([0]))
                    grp.compile(prog)
                    out = grp.run_ptrs(frames, records=records)
                else:
                    r = abi.DeviceRun(ctx, data, desc, n, records=records)
                    r.run()
                    out = r.fetch()
                    r.free()
            else:
                m = int(rng.integers(1, 4)) if form == "mapped" else int(rng.integers(2, 4))
                if m not in groups:
                    groups[m] = abi.Group([0] * m, flags=abi.OPT_GROUP_SHARED_DEVICE if m > 1 else 0)
                grp = groups[m]
                grp.compile(prog)
                out = (_mapped(grp, data, desc, n, records, _arena(arenas, m, grp), expect=dec, ctx=ctx)
                       if form == "mapped"
                       else grp.run_host(data, desc, records=records))
            _check(out, dec, n, npass, where)
            if records:
                bad = np.nonzero((out["records"][:n] != rec).any(axis=1))[0]
                assert len(bad) == 0, f"{where}: {len(bad)} records differ, first {bad[:5]}"
            rounds += 1
            print(f"ok round {rounds} {form} cfg {cfg} n {n} filters {len(prog)} records {records}", flush=True)
    finally:
        for a in arenas.values():
            a.close()
        for g in groups.values():
            g.close()
        ctx.close()
    assert rounds >= len(FORMS)


REGEX_POOL = ["GET", "[\\x00-\\x1f][a-z]", "^..?\\d", "MAG+IC", "a|b", "\\d\\d", "[^a-z]{3}", "(ab|cd)e",
              "x*y", "^$", ".", "HTTP/1\\.[01]", "[A-Z][a-z]+", "\\x00\\x00", "^\\w", "z$"]


@pytest.mark.skipif(not ol.ref_available(), reason="oracle/_ref (compiled reference) not built")
def test_randomized_payload_programs_vs_reference():
    """The same sweep with GPU PAYLOAD slots (regexes compiled to DFAs) between built-ins,
    checked against the compiled reference's own PacketFilter (std::regex per packet), on
    host, device-resident, zero-copy mapped and fixed-stride batches (C2's 64-B frames, whose
    LDS rows are 17 dwords). Runs BT_FUZZ_SECONDS / 3."""
    from golden_util import compare_decisions
    seconds = float(os.environ.get("BT_FUZZ_SECONDS", "15")) / 3
    seed0 = _seed() ^ 0x9A
    rng = np.random.default_rng(seed0)
    print(f"payload fuzz seed {seed0:#x}, {seconds:.0f} s", flush=True)
    ctx = abi.Context(0)
    grp = abi.Group([0, 0], flags=abi.OPT_GROUP_SHARED_DEVICE)
    arenas = {}
    t_end = time.time() + seconds
    rounds = 0
    try:
        while time.time() < t_end or rounds < 4:
            form = ("host", "device", "mapped", "fixed")[rounds % 4]
            cfg = [synth.C3, synth.C4, synth.FUZZ][int(rng.integers(0, 3))] if form != "fixed" else synth.C2
            n = int(rng.integers(1, 3000))
            data, desc = synth.capture(cfg, n, seed=int(rng.integers(1, 1 << 30)))
            if data.nbytes < 64:
                data = np.concatenate([data, np.zeros(64, np.uint8)])
            prog = random_programs(int(rng.integers(1, 1 << 30)), 1)[0]
            for k in range(int(rng.integers(1, 3))):
                prog.insert(int(rng.integers(0, len(prog) + 1)),
                            {"type": abi.PAYLOAD, "expr": REGEX_POOL[int(rng.integers(0, len(REGEX_POOL)))],
                             "priority": 40 + k})
            where = f"payload round {rounds} form {form} cfg {cfg} n {n} program {prog}"
            if form == "mapped":
                grp.compile(prog)
                out = _mapped(grp, data, desc, n, False, _arena(arenas, 2, grp))
            else:
                ctx.compile(prog)
                if form == "host":
                    out = ctx.run_host(data, desc, records=False)
                elif form == "fixed":   # no descriptors: frame i at i * 64
                    r = abi.DeviceRun(ctx, data[: n * 64], None, n, stride=64, records=False)
                    r.run()
                    out = r.fetch()
                    r.free()
                else:
                    r = abi.DeviceRun(ctx, data, desc, n, records=False)
                    r.run()
                    out = r.fetch()
                    r.free()
            code, src = ol.ref_filter(data, desc, n, prog)
            compare_decisions(out["decide"][:n], code, src, prog, where=where)
            rounds += 1
            print(f"ok payload round {rounds} {form} cfg {cfg} n {n} filters {len(prog)}", flush=True)
    finally:
        for a in arenas.values():
            a.close()
        grp.close()
        ctx.close()
