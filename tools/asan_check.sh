#!/bin/bash
# Host code of libbeatrice_gpu.so (filter compiler, ring walker/gather, DFA compiler,
# formatters, record unpacking, runtime) built with AddressSanitizer + UBSan, then the
# CPU test files that drive it without a GPU. Build container only (no GPU needed).
set -e
cd "$(dirname "$0")/../beatrice_amd/csrc"
OUT=${OUT:-/tmp/bt_asan}
mkdir -p $OUT
make -s obj/bt_kernels.o obj/bt_extract.o obj/bt_ring_walk.o
for f in bt_filter_compile bt_ring bt_regex_dfa bt_format; do
  g++ -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -fPIC -std=c++17 -I../../include -I. -c $f.cpp -o $OUT/$f.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -fPIC -std=c++17 -I../../include -I. -Xarch_host -fsanitize=address \
  -Xarch_host -fno-omit-frame-pointer -c bt_runtime.cpp -o $OUT/bt_runtime.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -fPIC -std=c++17 -I../../include -I. -Xarch_host -fsanitize=address \
  -Xarch_host -fno-omit-frame-pointer -c bt_group.cpp -o $OUT/bt_group.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libbeatrice_gpu.so obj/bt_kernels.o obj/bt_extract.o \
  obj/bt_ring_walk.o $OUT/bt_runtime.o $OUT/bt_group.o $OUT/bt_filter_compile.o $OUT/bt_ring.o $OUT/bt_regex_dfa.o \
  $OUT/bt_format.o -fsanitize=address,undefined
cd ../..
BT_LIB_PATH=$OUT/libbeatrice_gpu.so LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)" \
  ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  python -m pytest tests/test_format.py tests/test_abi.py tests/test_ring.py tests/test_filter_compile.py \
  tests/test_payload_dfa.py tests/test_sharding.py tests/test_extract_oracle.py tests/test_host_rules.py \
  -x -q -m "not gpu" -p no:cacheprovider
