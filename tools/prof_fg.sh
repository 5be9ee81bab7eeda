# Config 3 fun_and_grad_krylov_fun: timing (KT_EIG_STATS) and rocprofv3 kernel stats.
set -e
mkdir -p gpurun_out/fg
KT_EIG_STATS=2 timeout -k 10 200 python tools/prof_fg.py > gpurun_out/fg/run.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/fg/prof -o fg -- python3 $GRAFT_REPO_ROOT/tools/prof_fg.py > $GRAFT_REPO_ROOT/gpurun_out/fg/prof.log 2>&1
echo done
