set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_gridconv.py tests/test_gpu_gridnet.py tests/test_gpu_mono.py > gpurun_out/gt.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_mono.py --actors 64 --size 10 --arch gridnet --steps 10 \
  > gpurun_out/c2.log 2>&1 || exit $?
tail -1 gpurun_out/c2.log
bash tools/prof.sh prof_c2 tools/bench_mono.py --actors 64 --size 10 --arch gridnet --steps 4 --warmup 1 || exit $?
grep "at::native\|Cijk" gpurun_out/prof_c2_summary.md | cut -c1-200
