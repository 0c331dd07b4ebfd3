# The GPU suite, a settled bench, then kernel traces of the bench with and without the world-1
# collective rehearsal, and the rehearsal / timeline reports (profile 39, run as tag r5p).
#   bash tools/gpu_rehearsal.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
tag=$1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${tag}_gpu.log 2>&1 || { tail -40 gpurun_out/${tag}_gpu.log; exit 1; }
tail -3 gpurun_out/${tag}_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || { tail -20 gpurun_out/${tag}_bench.log; exit 2; }
tail -1 gpurun_out/${tag}_bench.log
cd /tmp && export TMPDIR=/tmp
for v in base reh; do
  extra=""; [ $v = reh ] && extra="--comm_rehearsal"
  timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/${tag}_$v -o run --output-format csv \
    -- python $R/bench.py --steps 30 --warmup 3 --settle 200 $extra > $R/gpurun_out/${tag}_$v.log 2>&1 || exit 3
  tail -1 $R/gpurun_out/${tag}_$v.log
done
python $R/tools/rehearsal_trace.py /tmp/${tag}_reh /tmp/${tag}_base > $R/gpurun_out/${tag}_rehearsal.txt 2>&1
python $R/tools/timeline.py /tmp/${tag}_reh > $R/gpurun_out/${tag}_timeline_reh.txt 2>&1
python $R/tools/timeline.py /tmp/${tag}_base > $R/gpurun_out/${tag}_timeline_base.txt 2>&1
cat $R/gpurun_out/${tag}_rehearsal.txt
