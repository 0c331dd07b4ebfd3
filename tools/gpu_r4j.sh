# Bench kernel timelines: launch-B head (default) vs head in launch A (MBK_ACT_FUSED=1).
#   bash tools/gpu_r4j.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4j}
export TMPDIR=/tmp
for f in 1 0; do
  rm -rf /tmp/${tag}_tl$f
  (cd /tmp && MBK_ACT_FUSED=$f timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/${tag}_tl$f -o run --output-format csv \
    -- python $R/bench.py --steps 12 --warmup 4) > gpurun_out/${tag}_tl_bench$f.log 2>&1 || { tail -5 gpurun_out/${tag}_tl_bench$f.log; exit 1; }
  python tools/timeline.py /tmp/${tag}_tl$f > gpurun_out/${tag}_timeline$f.txt 2>&1 || exit 2
  echo "== MBK_ACT_FUSED=$f"; head -12 gpurun_out/${tag}_timeline$f.txt
done
