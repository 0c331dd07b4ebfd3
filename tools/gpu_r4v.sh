# Learner update kernel trace of one BASELINE config (default: config 4, 24x24 IMPALA deep).
#   bash tools/gpu_r4v.sh <tag> [learner_only.py args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=${1:-r4v}; shift
LARGS=${@:---arch impala_deep --size 24}
export TMPDIR=/tmp
rm -rf /tmp/${tag}_lt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/${tag}_lt -o run --output-format csv \
  -- python $R/tools/learner_only.py $LARGS --steps 2) > gpurun_out/${tag}_lt.log 2>&1 || { tail -5 gpurun_out/${tag}_lt.log; exit 1; }
python tools/layer_times.py /tmp/${tag}_lt --out gpurun_out/${tag}_lt.md > /dev/null || exit 2
tail -1 gpurun_out/${tag}_lt.md
sort -t'|' -k4 -n -r gpurun_out/${tag}_lt.md | head -25
