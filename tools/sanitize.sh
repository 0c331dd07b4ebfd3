# Host-code sanitizer runs of the native runtime (GPU ASan / XNACK are not available on
# this pool, so only host code is instrumented). Usage: bash tools/sanitize.sh [asan|tsan|all]
set -eo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/microbeast_amd/csrc
OUT=${TMPDIR:-/tmp}/mbk_sanitize
mkdir -p $OUT
SRC="$C/tests/host_stress.cpp $C/runtime/shm_ring.cpp $C/runtime/vec_env.cpp $C/env/microrts_sim.cpp"
mode=${1:-all}
if [ "$mode" = asan ] || [ "$mode" = all ]; then
  g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined \
      -fno-sanitize-recover=undefined -I$C $SRC -o $OUT/host_stress_asan -lpthread
  ASAN_OPTIONS=detect_leaks=1 $OUT/host_stress_asan
fi
if [ "$mode" = tsan ] || [ "$mode" = all ]; then
  g++ -std=c++17 -O1 -g -fsanitize=thread -I$C $SRC -o $OUT/host_stress_tsan -lpthread
  TSAN_OPTIONS=halt_on_error=1 $OUT/host_stress_tsan
fi
