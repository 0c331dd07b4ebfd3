set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gridconv.py tests/test_gpu_gridnet.py > gpurun_out/gt.log 2>&1 || exit $?
tail -1 gpurun_out/gt.log
timeout -k 10 300 python bench.py --arch gridnet --size 10 --steps 10 --warmup 3 > gpurun_out/c2e.log 2>&1 || exit $?
tail -1 gpurun_out/c2e.log | cut -c1-400
bash tools/prof.sh prof_c2e bench.py --arch gridnet --size 10 --steps 4 --warmup 2 || exit $?
grep -c "at::native\|Cijk" gpurun_out/prof_c2e_summary.md
