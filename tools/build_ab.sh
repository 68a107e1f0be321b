# Builds an A/B variant of libbeatrice_gpu.so into beatrice_amd/ab/<name>/ with extra
# hipcc flags for bt_kernels.hip: bash tools/build_ab.sh NAME "-DFOO=1 ..."
set -e
NAME=$1; FLAGS=$2
D=beatrice_amd/ab/$NAME
mkdir -p $D
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Iinclude -Ibeatrice_amd/csrc"
$H $FLAGS -c beatrice_amd/csrc/bt_kernels.hip -o $D/bt_kernels.o
$H --offload-arch=gfx950 -shared -fPIC -o $D/libbeatrice_gpu.so $D/bt_kernels.o beatrice_amd/csrc/obj/bt_extract.o beatrice_amd/csrc/obj/bt_runtime.o beatrice_amd/csrc/obj/bt_filter_compile.o beatrice_amd/csrc/obj/bt_ring.o beatrice_amd/csrc/obj/bt_regex_dfa.o beatrice_amd/csrc/obj/bt_format.o
rm -f $D/bt_kernels.o
echo built $D
