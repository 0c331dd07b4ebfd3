# Kernel-trace + stats profile of one command on the GPU box, summarised to markdown.
#   bash tools/prof.sh <name> <python args...>
# writes gpurun_out/<name>.log (program output) and gpurun_out/<name>_summary.md
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
name=$1; shift
script=$1; shift
case $script in /*) ;; *) script=$R/$script ;; esac  # prof runs from /tmp
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/$name -o run --output-format csv \
  -- python "$script" "$@" > $R/gpurun_out/$name.log 2>&1 || exit $?
python $R/tools/rocprof_summary.py /tmp/$name $R/gpurun_out/${name}_summary.md --drop-trace ${MBK_PROF_SEQ:+--seq=$MBK_PROF_SEQ}
