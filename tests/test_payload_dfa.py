"""CPU: the PAYLOAD regex -> byte-DFA compiler (beatrice_amd/csrc/bt_regex_dfa.cpp,
SURVEY §8(f) 3), checked without a GPU:

  * against std::regex_search itself — the libstdc++ function the reference's
    applyPayloadFilter calls — by the differential fuzzer tests/cpp/test_regex_dfa
    (random patterns over the modelled ECMAScript subset x random byte strings, plus
    the applyPayloadFilter window on synthetic frames);
  * against the compiled reference's PacketFilter outcomes in the goldens: every
    single-PAYLOAD-filter set on every capture, through the host executor of the
    same DFA blob the kernel runs."""
import os
import subprocess

import numpy as np
import pytest

from beatrice_amd import abi, synth
from conftest import GOLDEN, load_golden

FUZZ_BIN = os.path.join(os.path.dirname(GOLDEN), "cpp", "test_regex_dfa")


def test_dfa_fuzz_against_std_regex():
    assert os.path.exists(FUZZ_BIN), "tests/cpp/test_regex_dfa not built (make -C tests/cpp)"
    r = subprocess.run([FUZZ_BIN, "200", "60", "4242"], capture_output=True, text=True, timeout=600)
    print(r.stdout[-2000:])
    assert r.returncode == 0 and "ALL OK" in r.stdout, r.stdout[-3000:]


def _single_payload_sets(man, cap):
    for s in man["captures"][cap]["filter_sets"]:
        fs = man["filter_sets"][s]
        if len(fs) == 1 and fs[0]["type"] == abi.PAYLOAD and fs[0]["expr"]:
            yield s, fs[0]["expr"]


@pytest.mark.parametrize("cap", ["http", "edge", "fuzz", "c3"])
def test_dfa_matches_reference_goldens(cap):
    g, man = load_golden(cap)
    data, desc = g["data"], g["desc"]
    off, ln = synth.desc_off(desc), synth.desc_len(desc)
    checked = 0
    for s, expr in _single_payload_sets(man, cap):
        try:
            blob = abi.payload_dfa(expr)
        except abi.BtError:
            assert np.all(g[f"code__{s}"] == 1), f"{s}: std::regex rejects {expr!r}, the reference never passes"
            continue
        if blob is None:
            continue   # outside the subset: stays on the host
        want = g[f"code__{s}"] == 0
        got = np.array([abi.payload_dfa_eval(blob, data[o:o + n]) for o, n in zip(off, ln)])
        bad = np.nonzero(got != want)[0]
        assert len(bad) == 0, f"{cap}/{s} /{expr}/: {len(bad)} frames differ, first {bad[:5]}"
        checked += 1
    assert checked >= (10 if cap in ("http", "edge", "fuzz") else 1)


def test_subset_classification():
    on_gpu = ["GET", "GET|POST", "^GET /", "HTTP/1\\.[01]", "[^]", "[]", "^$", "a|", "x{0}y", "\\0", "(?:a|b)*c",
              "[\\x80-\\xff]{4,}", "\\s+$", "a**", "a{2,3}?"]
    on_host = ["\\bfoo", "(ab)\\1", "(?=a)b", "[[:alpha:]]", "\\cA", "\\u0041", "\\a", "(a|b)*a(a|b){12}"]
    rejected = ["[", "a{2,1}", "(", "\\1", "[z-a]", "{"]
    for e in on_gpu:
        assert abi.payload_dfa(e) is not None, e
    for e in on_host:
        assert abi.payload_dfa(e) is None, e
    for e in rejected:
        with pytest.raises(abi.BtError):
            abi.payload_dfa(e)


def test_host_compile_keeps_payload_on_host_kind():
    """bt_filter_compile_host has no context (no DFA pool): PAYLOAD stays BT_K_HOST there;
    the GPU kind is assigned by bt_filter_compile on a context (tests/test_gpu_payload.py)."""
    slots = abi.compile_host([{"type": abi.PAYLOAD, "expr": "GET", "priority": 1}])
    assert [abi.KINDS[s.kind] for s in slots] == ["HOST"]
