# Bench kernel timeline (policy steps under / outside the learner) -> profiles material.
#   bash tools/gpu_r4e.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4e}
export TMPDIR=/tmp
rm -rf /tmp/${tag}_tl
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/${tag}_tl -o run --output-format csv \
  -- python $R/bench.py --steps 12 --warmup 4) > gpurun_out/${tag}_tl_bench.log 2>&1 || { tail -5 gpurun_out/${tag}_tl_bench.log; exit 1; }
python tools/timeline.py /tmp/${tag}_tl > gpurun_out/${tag}_timeline.txt 2>&1 || exit 2
cat gpurun_out/${tag}_timeline.txt | head -30
