"""CPU: the synthetic capture generator is deterministic and matches SURVEY §8(d)."""
import numpy as np

from beatrice_amd import synth


def test_deterministic_and_seeded():
    a = synth.capture(synth.C3, 5000)
    b = synth.capture(synth.C3, 5000, threads=1)
    c = synth.capture(synth.C3, 5000, seed=1)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert not np.array_equal(a[0][:4096], c[0][:4096])


def test_layouts():
    d2, c2 = synth.capture(synth.C2, 1000)
    assert np.all(synth.desc_len(c2) == 64) and np.all(synth.desc_off(c2) == np.arange(1000) * 64)
    _, c3 = synth.capture(synth.C3, 20000)
    ln = synth.desc_len(c3)
    assert set(np.unique(ln).tolist()) == {64, 512, 1500}
    frac = [np.mean(ln == v) for v in (64, 512, 1500)]
    assert abs(frac[0] - 7 / 12) < 0.02 and abs(frac[1] - 4 / 12) < 0.02
    assert np.all(synth.desc_off(c3) % 64 == 0)
    d4, c4 = synth.capture(synth.C4, 20000)
    assert np.all(synth.desc_off(c4) % 4 == 2)
    ln4 = synth.desc_len(c4)
    assert ln4.min() >= 64 and ln4.max() <= 1500 + 4 * 15 + 60
    # frames never overlap
    off = synth.desc_off(c4)
    assert np.all(off[1:] >= off[:-1] + ln4[:-1])


def test_c2_headers():
    d, c = synth.capture(synth.C2, 256)
    f = d[:256 * 64].reshape(256, 64)
    assert np.all(f[:, 12] == 0x08) and np.all(f[:, 13] == 0x00) and np.all(f[:, 14] == 0x45)
    assert np.all(f[:, 23] == 17) and np.all(f[:, 26] == 10) and np.all(f[:, 30] == 192)
    dport = f[:, 36].astype(int) * 256 + f[:, 37]
    assert dport.max() < 4096
