"""CPU: the oracle's decisions on seeded random PacketFilter programs (tests/random_programs.py)
against the compiled reference's applyFilters on the same frames: pins the checker the GPU
test (tests/test_gpu_parity.py::test_random_programs_match_oracle) compares with."""
import pytest

import oracle_lib as ol
from beatrice_amd import synth
from golden_util import compare_decisions
from random_programs import random_programs

pytestmark = pytest.mark.skipif(not ol.ref_available(), reason="oracle/_ref not built")


@pytest.mark.parametrize("cfg", [synth.FUZZ, synth.C3])
def test_oracle_matches_reference_on_random_programs(cfg):
    n = 4000
    data, desc = synth.capture(cfg, n, seed=0x5A + cfg)
    for i, prog in enumerate(random_programs(0xF117E2 + cfg, 40)):
        _, dec, _ = ol.oracle_run(data, desc, n, prog, parse=False, threads=2)
        code, src = ol.ref_filter(data, desc, n, prog)
        host = compare_decisions(dec, code, src, prog, where=f"program {i}: {prog}")
        assert len(host) == 0, f"program {i}: built-in kinds never go to the host"
