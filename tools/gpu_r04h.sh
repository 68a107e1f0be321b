# round 4: the plugin fed hot frames, BEATRICE_GPU_PACK off / on (alternating processes, one box);
# small calls again with the final threshold
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
bash tools/ab_cmd.sh $O/pack 2 "pack0|BEATRICE_GPU_PACK=0|" "pack1|BEATRICE_GPU_PACK=1|" -- tools/surfaces/surface_bench plugin-hot --seconds 2 || exit 1
timeout -k 10 300 tools/surfaces/surface_bench single --seconds 1 > $O/surf_single.jsonl 2> $O/surf_single.err || exit 1
echo ALL-DONE
