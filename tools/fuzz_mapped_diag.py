"""Root-cause harness for the mapped-path differences of test_randomized_parity_sweep.

Runs the suite's sweep (tests/test_gpu_fuzz.py, same seed, same forms) with per-round
registration (the round-5 form that showed the difference) and, when a mapped round's
decisions differ from the oracle, examines the round while its buffers are still registered:

  rerun     the same bt_group_parse_filter_mapped call again (outputs poisoned 0xFF first)
  view      the device's own copy of the capture bytes through the same alias (the extract
            kernel's image output), compared with the host bytes: which byte ranges differ, and
            what the device read there (zeros, bytes of an earlier round's buffer, ...)
  history   every buffer registered / device buffer allocated in the last rounds: host
            range, its pages, its device alias, so a reused address (host page, alias VA or
            hipMalloc VA) is visible
  fresh     unregister + register the capture again, run again

Writes one JSON object per finding to stdout; the sweep's own lines go to stderr.
Usage: python tools/fuzz_mapped_diag.py [--seconds S] [--seed 0xB1A5] [--keep-going N]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from beatrice_amd import abi  # noqa: E402
import test_gpu_fuzz as tf  # noqa: E402
import reg_probe as rp  # noqa: E402

PAGE = 4096
hip = rp.Hip()
history = []          # (round, what, host_lo, nbytes, alias)
state = {"round": 0, "pending": None, "found": 0, "mapped_rounds": 0}
_orig_buf_init = abi.DeviceBuffer.__init__


def _buf_init(self, ctx, nbytes):
    _orig_buf_init(self, ctx, nbytes)
    history.append((state["round"], "hipMalloc", None, int(nbytes), int(self.ptr)))


abi.DeviceBuffer.__init__ = _buf_init


def alias_of(p: int) -> int:
    d = ctypes.c_void_p(0)
    rc = hip.L.hipHostGetDevicePointer(ctypes.byref(d), p, 0)
    return d.value if rc == 0 else -rc


def mapped(grp, data, desc, n, records, arena=None):
    """tf._mapped's per-round form, leaving the buffers registered until check()."""
    state["mapped_rounds"] += 1
    tiles = max(1, (n + 63) // 64)
    pidx = np.zeros(max(n, 1), np.uint32)
    npass = np.zeros(1, np.uint32)
    h_rec = np.zeros(tiles * 6144, np.uint8) if records else None
    h_dec = np.zeros(tiles * 64, np.uint8)
    h_ver = np.zeros(tiles, np.uint64)
    held = [a for a in (data, desc, h_rec, h_dec, h_ver) if a is not None]
    names = ["data", "desc", "rec", "dec", "ver"] if records else ["data", "desc", "dec", "ver"]
    for nm, a in zip(names, held):
        grp.register(a)
        history.append((state["round"], nm, a.ctypes.data, a.nbytes, alias_of(a.ctypes.data)))
    batch = abi.Batch(data.ctypes.data, desc.ctypes.data, 0, n, data.nbytes, abi.DESC_PACKED, 0)
    outs = abi.Outputs(None if h_rec is None else h_rec.ctypes.data, n, h_ver.ctypes.data, h_dec.ctypes.data,
                       pidx.ctypes.data, npass.ctypes.data)
    grp.run_mapped(batch, outs)
    state["pending"] = dict(grp=grp, held=held, batch=batch, outs=outs, data=data, desc=desc, n=n,
                            h_dec=h_dec, h_ver=h_ver, h_rec=h_rec, pidx=pidx, npass=npass)
    return {"decide": h_dec[:n].copy(), "verdict": h_ver.copy(), "pass_idx": pidx[:int(npass[0])].copy(),
            "n_pass": int(npass[0]), "records": abi.untile_records(h_rec, n) if records else None}


def release():
    p, state["pending"] = state["pending"], None
    if p:
        for a in p["held"]:
            p["grp"].unregister(a)


def ranges(mask: np.ndarray):
    idx = np.nonzero(mask)[0]
    if not len(idx):
        return []
    cuts = np.nonzero(np.diff(idx) > 1)[0]
    starts = np.concatenate([[idx[0]], idx[cuts + 1]])
    ends = np.concatenate([idx[cuts], [idx[-1]]]) + 1
    return [(int(s), int(e)) for s, e in zip(starts, ends)]


def diagnose(out, dec, n, where):
    p = state["pending"]
    data, desc = p["data"], p["desc"]
    bad = np.nonzero(out["decide"][:n] != dec)[0]
    from beatrice_amd import synth
    off = synth.desc_off(desc).astype(np.int64)
    ln = synth.desc_len(desc).astype(np.int64)
    rep = {"where": where, "round": state["round"], "n_bad": int(len(bad)), "bad_first": bad[:40].tolist(),
           "got": out["decide"][bad[:40]].tolist(), "want": dec[bad[:40]].tolist(),
           "bad_frame_bytes": [[int(off[i]), int(off[i] + ln[i])] for i in bad[:10]],
           "data": {"host": hex(data.ctypes.data), "nbytes": int(data.nbytes), "alias": hex(alias_of(data.ctypes.data))},
           "dec_arr": {"host": hex(p["h_dec"].ctypes.data), "alias": hex(alias_of(p["h_dec"].ctypes.data))}}
    # rerun on the same registrations
    p["h_dec"].fill(0xFF)
    p["h_ver"].fill(0xFFFFFFFFFFFFFFFF)
    p["grp"].run_mapped(p["batch"], p["outs"])
    rep["rerun_bad"] = int(np.count_nonzero(p["h_dec"][:n] != dec))
    # the device's view of the capture through the same alias
    a = alias_of(data.ctypes.data)
    nb = data.nbytes // 256 * 256
    if a > 0 and nb:
        ctx = tf._diag_ctx
        view = rp.gpu_view(ctx, a, nb)
        diff = view[:nb] != data[:nb]
        rr = ranges(diff)
        rep["view_diff_ranges"] = rr[:20]
        rep["view_diff_bytes"] = int(diff.sum())
        if rr:
            s, e = rr[0]
            rep["view_sample"] = {"host": data[s:min(e, s + 32)].tolist(), "dev": view[s:min(e, s + 32)].tolist(),
                                  "dev_zero_frac": float((view[s:e] == 0).mean())}
            pg0, pg1 = (data.ctypes.data + s) // PAGE, (data.ctypes.data + e - 1) // PAGE
            rep["view_diff_pages"] = [hex(pg0 * PAGE), hex(pg1 * PAGE), int(pg1 - pg0 + 1)]
            lo_h, hi_h = pg0 * PAGE, (pg1 + 1) * PAGE
            lo_a, hi_a = a + (lo_h - data.ctypes.data), a + (hi_h - data.ctypes.data)
            hits = []
            for (r, what, host, nbytes, al) in history[:-8]:
                h_hit = host is not None and host < hi_h and host + nbytes > lo_h
                a_hit = al is not None and al > 0 and al < hi_a and al + nbytes > lo_a
                if h_hit or a_hit:
                    hits.append({"round": r, "what": what, "host": hex(host) if host else None, "nbytes": nbytes,
                                 "alias": hex(al) if al and al > 0 else al, "host_overlap": h_hit, "alias_overlap": a_hit})
            rep["history_overlaps"] = hits[-30:]
    # the descriptors through their alias (a zero descriptor reads as an empty frame)
    ad = alias_of(desc.ctypes.data)
    ndb = desc.nbytes // 256 * 256
    if ad > 0 and ndb:
        dview = rp.gpu_view(tf._diag_ctx, ad, ndb)
        dd = dview[:ndb] != desc.view(np.uint8)[:ndb]
        rep["desc_view_diff_ranges"] = ranges(dd)[:20]
        rep["desc_view_diff_bytes"] = int(dd.sum())
    rep["desc_arr"] = {"host": hex(desc.ctypes.data), "nbytes": int(desc.nbytes), "alias": hex(ad)}
    # a fresh registration of the capture
    grp = p["grp"]
    grp.unregister(data)
    grp.register(data)
    rep["fresh_alias"] = hex(alias_of(data.ctypes.data))
    p["h_dec"].fill(0xFF)
    grp.run_mapped(p["batch"], p["outs"])
    rep["fresh_bad"] = int(np.count_nonzero(p["h_dec"][:n] != dec))
    print(json.dumps(rep), file=state["out"], flush=True)


def check(out, dec, n, npass, where):
    try:
        if state["pending"] is not None and np.count_nonzero(out["decide"][:n] != dec):
            state["found"] += 1
            diagnose(out, dec, n, where)
            if state["found"] >= state["max"]:
                raise SystemExit(0)
            return
        tf._orig_check(out, dec, n, npass, where)
    finally:
        release()
        state["round"] += 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--seed", default="0xB1A5")
    ap.add_argument("--keep-going", type=int, default=3, help="stop after this many differing rounds")
    a = ap.parse_args()
    os.environ["BT_FUZZ_SECONDS"] = str(a.seconds)
    os.environ["BT_FUZZ_SEED"] = a.seed
    os.environ["BT_FUZZ_REGISTER_EACH"] = "1"
    state["max"] = a.keep_going
    tf._orig_check = tf._check
    tf._check = check
    tf._mapped = mapped
    tf._diag_ctx = abi.Context(0)
    state["out"] = real = sys.stdout
    sys.stdout = sys.stderr
    t0 = time.time()
    try:
        tf.test_randomized_parity_sweep()
    except SystemExit:
        pass
    finally:
        sys.stdout = real
        print(json.dumps({"rounds": state["round"], "mapped_rounds": state["mapped_rounds"], "found": state["found"],
                          "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
