# round 4 closing evidence, one box: the end-to-end paths (host gather, zero-copy, TPACKET_V3 ring in
# place / packed gather every 2nd batch in place, groups of 2 and 4 sharing the device, the
# sparse-frame host gather option) for C2 / C3 / C4
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r04e2e} STEPS="e2e" E2E_CFGS="c2 c3 c4" \
  E2E_MODES=" ;--zero-copy;--tpacket;--tpacket --gather --dense --mix 2;--group 2;--group 4;--group 1 --flags 0x10000" \
  bash tools/gpu_round.sh
