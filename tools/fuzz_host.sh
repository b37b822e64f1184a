#!/bin/bash
# Host-side fuzzing of the asset readers under AddressSanitizer + UBSan (CPU only):
#   ITERS=3000 bash tools/fuzz_host.sh
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/fuzz_host_build
mkdir -p $B
C=$R/metal4-raytracing_amd/csrc
g++ -std=c++17 -O1 -g -fsanitize=address,undefined,float-cast-overflow -fno-sanitize-recover=undefined,float-cast-overflow -ffp-contract=off \
    -I$R/include -o $B/fuzz_host $R/tools/fuzz_host.cpp $C/rt_scene.cpp $C/rt_bvh.cpp $C/rt_texture.cpp \
    $C/rt_usd.cpp -lz -lpthread
python3 $R/tools/fuzz_seeds.py $B/seeds > /dev/null
for m in usda usdc usdz png obj; do
  ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
    $B/fuzz_host $m $B/seeds/seed.$m ${ITERS:-3000} ${SEED:-1}
done
# internal-reference fan-out over a large array (fewer iterations: each input is ~100 KB)
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
  $B/fuzz_host usda $B/seeds/seed_fanout.usda $(( ${ITERS:-3000} / 10 + 1 )) ${SEED:-1}
