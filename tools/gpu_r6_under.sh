# kernel trace of the headline bench + which learner kernel each acting launch ran under:
#   bash tools/gpu_r6_under.sh <tag> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/$tag -o run --output-format csv \
  -- python $R/bench.py --steps 20 --warmup 5 "$@" > $R/gpurun_out/$tag.log 2>&1 || exit $?
python $R/tools/acting_under.py /tmp/$tag 0.5 > $R/gpurun_out/${tag}_under.md && cat $R/gpurun_out/${tag}_under.md
grep metric $R/gpurun_out/$tag.log | cut -c1-200
