# Builds an A/B variant of libbeatrice_gpu.so into beatrice_amd/ab/<name>/:
#   bash tools/build_ab.sh NAME "<hipcc flags for bt_kernels.hip>" ["<g++ flags for bt_ring.cpp>"]
# Every other object comes from beatrice_amd/csrc/obj (make -C beatrice_amd/csrc first). Load
# the variant with BT_LIB_PATH (Python) or LD_LIBRARY_PATH (the C++ tools).
set -e
NAME=$1; FLAGS=$2; RING_FLAGS=$3
D=beatrice_amd/ab/$NAME
O=beatrice_amd/csrc/obj
mkdir -p $D
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Iinclude -Ibeatrice_amd/csrc"
$H $FLAGS -c beatrice_amd/csrc/bt_kernels.hip -o $D/bt_kernels.o
g++ -O2 -fPIC -std=c++17 -Wall -Iinclude -Ibeatrice_amd/csrc $RING_FLAGS -c beatrice_amd/csrc/bt_ring.cpp -o $D/bt_ring.o
$H -shared -fPIC -o $D/libbeatrice_gpu.so $D/bt_kernels.o $D/bt_ring.o $O/bt_extract.o $O/bt_ring_walk.o \
    $O/bt_runtime.o $O/bt_filter_compile.o $O/bt_ring_stage.o $O/bt_regex_dfa.o $O/bt_format.o $O/bt_group.o \
    $O/bt_pin.o
rm -f $D/bt_kernels.o $D/bt_ring.o
echo built $D
