# conv0_row padded-row skip test, GridNet learner / engine, learner with / without bitmap rows.
#   bash tools/gpu_r4h.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4h}
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_gridnet.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 300 python tools/learner_only.py --arch gridnet --size 10 --steps 3 > gpurun_out/${tag}_gn_learner.log 2>&1 || exit 2
tail -1 gpurun_out/${tag}_gn_learner.log
for v in "" "--no_abits"; do
  timeout -k 10 300 python tools/learner_only.py --steps 5 $v > gpurun_out/${tag}_learner$v.log 2>&1 || exit 3
  echo "learner $v: $(tail -1 gpurun_out/${tag}_learner$v.log)"
done
bash tools/lt_ab.sh ${tag} "MBK_NOP=0" || exit 4
grep -E "head_count|head_scatter|update span" gpurun_out/${tag}_lt1.md
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --size 10 --arch gridnet > gpurun_out/${tag}_c2e.log 2>&1 || exit 5
echo "c2 engine: $(tail -1 gpurun_out/${tag}_c2e.log | cut -c1-160)"
