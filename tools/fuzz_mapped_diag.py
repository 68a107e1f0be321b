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
page_sums = []        # (round, host_lo, first whole page address, per-page word sums) of the last captures


def _page_sums(a: np.ndarray):
    """Per-page sums of the whole pages inside a (absolute page addresses from p0): a page's
    content fingerprint, to recognise which earlier capture a stale device page holds."""
    lo = a.ctypes.data
    p0 = (lo + PAGE - 1) // PAGE * PAGE
    k = max(0, (lo + a.nbytes - p0) // PAGE)
    b = np.frombuffer(a, np.uint8, count=a.nbytes)[p0 - lo:p0 - lo + k * PAGE]
    return p0, b.view(np.uint64).reshape(k, PAGE // 8).sum(axis=1, dtype=np.uint64) if k else np.zeros(0, np.uint64)


def _whose(view_sums: np.ndarray, p0: int, stale: np.ndarray) -> list:
    """For each stale page (index into view_sums, absolute page p0 + i*PAGE): the most recent
    earlier capture whose page at the SAME address held exactly what the device read, else any
    earlier capture's page anywhere with that content."""
    out = []
    for i in stale[:16]:
        addr, want = p0 + int(i) * PAGE, view_sums[i]
        hit = None
        for (r, lo, q0, sums) in reversed(page_sums[:-1]):
            j = (addr - q0) // PAGE
            if 0 <= j < len(sums) and sums[j] == want:
                hit = {"page": hex(addr), "same_address": True, "round": r, "capture_base": hex(lo)}
                break
        if hit is None:
            for (r, lo, q0, sums) in reversed(page_sums[:-1]):
                j = np.nonzero(sums == want)[0]
                if len(j):
                    hit = {"page": hex(addr), "same_address": False, "round": r, "capture_base": hex(lo),
                           "at": hex(q0 + int(j[0]) * PAGE)}
                    break
        out.append(hit or {"page": hex(addr), "unknown": True, "zero": bool(want == 0)})
    return out
state = {"round": 0, "found": 0, "mapped_rounds": 0, "form": "r05", "history": True, "thp": "default"}
_orig_buf_init = abi.DeviceBuffer.__init__


def _buf_init(self, ctx, nbytes):
    _orig_buf_init(self, ctx, nbytes)
    history.append((state["round"], "hipMalloc", None, int(nbytes), int(self.ptr)))


abi.DeviceBuffer.__init__ = _buf_init


def alias_of(p: int) -> int:
    d = ctypes.c_void_p(0)
    rc = hip.L.hipHostGetDevicePointer(ctypes.byref(d), p, 0)
    return d.value if rc == 0 else -rc


def _host_array(shape, dtype=np.uint8):
    """abi.host_array, with MADV_HUGEPAGE on its mapping under --thp on."""
    a = abi.host_array(shape, dtype)
    if state["thp"] == "on":
        import mmap
        b = a
        while not isinstance(b, mmap.mmap):
            b = b.obj if isinstance(b, memoryview) else b.base
        b.madvise(mmap.MADV_HUGEPAGE)
    return a


def _host_copy(arr):
    out = _host_array(arr.shape, arr.dtype)
    np.copyto(out, arr)
    return out


def mapped(grp, data, desc, n, records, arena=None, expect=None, ctx=None):
    """tf._mapped's per-round form. --form r05: the round-5 sweep's buffers (the capture arrays
    as synth made them, np.zeros outputs: heap or mmap chunks as glibc places them, possibly
    sharing pages); --form pages: every buffer on pages of its own (abi.host_copy /
    host_array, the current sweep). Unregistered right after the call, as both sweeps do; a
    round whose decisions differ is examined first, while its buffers are still registered."""
    state["mapped_rounds"] += 1
    tiles = max(1, (n + 63) // 64)
    pidx = np.zeros(max(n, 1), np.uint32)
    npass = np.zeros(1, np.uint32)
    if state["form"] == "pages":
        mk = _host_array
        data, desc = _host_copy(data), _host_copy(desc)
    else:
        mk = np.zeros
    h_rec = mk(tiles * 6144, np.uint8) if records else None
    h_dec = mk(tiles * 64, np.uint8)
    h_ver = mk(tiles, np.uint64)
    if state["form"] == "pages":
        h_dec.fill(0xFF)
        h_ver.fill(0xFFFFFFFFFFFFFFFF)
    held = [a for a in (data, desc, h_rec, h_dec, h_ver) if a is not None]
    names = ["data", "desc", "rec", "dec", "ver"] if records else ["data", "desc", "dec", "ver"]
    for nm, a in zip(names, held):
        grp.register(a)
        history.append((state["round"], nm, a.ctypes.data, a.nbytes,
                        alias_of(a.ctypes.data) if state["history"] else None))
        if nm == "data":
            page_sums.append((state["round"], a.ctypes.data, *_page_sums(a)))
            del page_sums[:-400]
        del history[:-4000]
    batch = abi.Batch(data.ctypes.data, desc.ctypes.data, 0, n, data.nbytes, abi.DESC_PACKED, 0)
    outs = abi.Outputs(None if h_rec is None else h_rec.ctypes.data, n, h_ver.ctypes.data, h_dec.ctypes.data,
                       pidx.ctypes.data, npass.ctypes.data)
    rep = None
    try:
        grp.run_mapped(batch, outs)
        out = {"decide": h_dec[:n].copy(), "verdict": h_ver.copy(), "pass_idx": pidx[:int(npass[0])].copy(),
               "n_pass": int(npass[0]), "records": abi.untile_records(h_rec, n) if records else None}
        last = state.get("last_oracle")
        rec_bad = bool(records and last is not None and last[0] is not None and len(last[0]) == n
                       and np.count_nonzero((out["records"][:n] != last[0]).any(axis=1)))
        if expect is not None and (np.count_nonzero(out["decide"] != expect) or rec_bad):
            state["found"] += 1
            rep = diagnose(out, expect, n, dict(grp=grp, batch=batch, outs=outs, data=data, desc=desc,
                                                h_dec=h_dec, h_ver=h_ver, names=names, held=held))
    finally:
        for a in held:
            grp.unregister(a)
    if rep is not None:
        # after the unregister: the same capture registered afresh
        for a in held:
            grp.register(a)
        h_dec.fill(0xFF)
        try:
            grp.run_mapped(batch, outs)
            rep["fresh_bad"] = int(np.count_nonzero(h_dec[:n] != expect))
        finally:
            for a in held:
                grp.unregister(a)
        out["evidence"] = rep
    return out


def ranges(mask: np.ndarray):
    idx = np.nonzero(mask)[0]
    if not len(idx):
        return []
    cuts = np.nonzero(np.diff(idx) > 1)[0]
    starts = np.concatenate([[idx[0]], idx[cuts + 1]])
    ends = np.concatenate([idx[cuts], [idx[-1]]]) + 1
    return [(int(s), int(e)) for s, e in zip(starts, ends)]


def diagnose(out, dec, n, p):
    data, desc = p["data"], p["desc"]
    bad = np.nonzero(out["decide"][:n] != dec)[0]
    from beatrice_amd import synth
    off = synth.desc_off(desc).astype(np.int64)
    ln = synth.desc_len(desc).astype(np.int64)
    rep = {"round": state["round"], "n_bad": int(len(bad)), "bad_first": bad[:40].tolist(),
           "got": out["decide"][bad[:40]].tolist(), "want": dec[bad[:40]].tolist(),
           "bad_frame_bytes": [[int(off[i]), int(off[i] + ln[i])] for i in bad[:10]],
           "arrays": {nm: {"host": hex(a.ctypes.data), "nbytes": int(a.nbytes), "page_off": a.ctypes.data % PAGE,
                           "alias": hex(alias_of(a.ctypes.data))} for nm, a in zip(p["names"], p["held"])}}
    lo = [a.ctypes.data // PAGE for a in p["held"]]
    hi = [(a.ctypes.data + a.nbytes - 1) // PAGE for a in p["held"]]
    rep["shared_pages"] = [[p["names"][i], p["names"][j]] for i in range(len(lo)) for j in range(i + 1, len(lo))
                           if lo[i] <= hi[j] and lo[j] <= hi[i]]
    # the device's view of the capture and its descriptors through the same aliases, before the rerun
    for nm, arr in (("data", data), ("desc", desc.view(np.uint8))):
        a = alias_of(arr.ctypes.data)
        nb = arr.nbytes // 256 * 256
        if a <= 0 or not nb:
            rep[nm + "_view"] = "no alias" if a <= 0 else "short"
            continue
        view = rp.gpu_view(tf._diag_ctx, a, nb)
        diff = view[:nb] != arr[:nb]
        rr = ranges(diff)
        v = {"diff_bytes": int(diff.sum()), "diff_ranges": rr[:20]}
        if rr:
            s0, e0 = rr[0]
            v["sample_host"] = arr[s0:min(e0, s0 + 32)].tolist()
            v["sample_dev"] = view[s0:min(e0, s0 + 32)].tolist()
            v["dev_zero_frac"] = float((view[:nb][diff] == 0).mean())
            pg0, pg1 = (arr.ctypes.data + s0) // PAGE, (arr.ctypes.data + rr[-1][1] - 1) // PAGE
            v["pages"] = [hex(pg0 * PAGE), hex(pg1 * PAGE), int(pg1 - pg0 + 1)]
            lo_h, hi_h = pg0 * PAGE, (pg1 + 1) * PAGE
            hits = []
            for (r, what, host, nbytes, al) in history[:-len(p["held"])]:
                if host is not None and host < hi_h and host + nbytes > lo_h:
                    hits.append({"round": r, "what": what, "host": hex(host), "nbytes": nbytes,
                                 "alias": hex(al) if al and al > 0 else al})
            v["history_host_overlaps"] = hits[-30:]
        if nm == "data":
            p0, hs = _page_sums(arr)
            off0 = p0 - arr.ctypes.data
            k = len(hs)
            vb = view[off0:off0 + k * PAGE]
            k = len(vb) // PAGE
            vs = vb[:k * PAGE].view(np.uint64).reshape(k, PAGE // 8).sum(axis=1, dtype=np.uint64)
            stale = np.nonzero(vs != hs[:k])[0]
            v["stale_pages"] = {"n": int(len(stale)), "first": hex(p0 + int(stale[0]) * PAGE) if len(stale) else None,
                                "runs": ranges(vs != hs[:k])[:10], "whose": _whose(vs, p0, stale)}
        rep[nm + "_view"] = v
    # the same call again on the same registrations
    p["h_dec"].fill(0xFF)
    p["h_ver"].fill(0xFFFFFFFFFFFFFFFF)
    p["grp"].run_mapped(p["batch"], p["outs"])
    rep["rerun_bad"] = int(np.count_nonzero(p["h_dec"][:n] != dec))
    rep["rerun_got"] = p["h_dec"][bad[:40]].tolist()
    return rep


def check(out, dec, n, npass, where):
    try:
        ev = out.get("evidence") if isinstance(out, dict) else None
        if ev is not None:
            ev["where"] = where
            print(json.dumps(ev), file=state["out"], flush=True)
            if state["found"] >= state["max"]:
                raise SystemExit(0)
            return
        tf._orig_check(out, dec, n, npass, where)
    finally:
        state["round"] += 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120)
    ap.add_argument("--seed", default="0xB1A5")
    ap.add_argument("--keep-going", type=int, default=3, help="stop after this many differing rounds")
    ap.add_argument("--form", choices=("r05", "pages"), default="r05")
    ap.add_argument("--thp", choices=("default", "off", "on"), default="default",
                    help="off: numpy's MADV_HUGEPAGE hint on large arrays disabled; on: --form pages "
                         "buffers madvised MADV_HUGEPAGE")
    ap.add_argument("--no-history", action="store_true", help="no device-pointer lookup per registration")
    a = ap.parse_args()
    state["form"] = a.form
    state["thp"] = a.thp
    if a.thp == "off":
        try:
            from numpy._core.multiarray import _set_madvise_hugepage
        except ImportError:
            from numpy.core.multiarray import _set_madvise_hugepage
        _set_madvise_hugepage(False)
    import oracle_lib as ol
    _orun = ol.oracle_run

    def oracle_run(*args, **kw):   # the sweep's expected records, for the evidence hook
        r = _orun(*args, **kw)
        state["last_oracle"] = r
        return r
    ol.oracle_run = oracle_run
    tf.ol.oracle_run = oracle_run
    state["history"] = not a.no_history
    os.environ["BT_FUZZ_SECONDS"] = str(a.seconds)
    os.environ["BT_FUZZ_SEED"] = a.seed
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
    except AssertionError as e:   # a difference the evidence hook does not cover (records): report it
        print(json.dumps({"assertion": str(e)[:3000]}), file=real, flush=True)
    finally:
        sys.stdout = real
        print(json.dumps({"form": state["form"], "thp": state["thp"], "lib": abi.LIB_PATH, "rounds": state["round"], "mapped_rounds": state["mapped_rounds"], "found": state["found"],
                          "seconds": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
