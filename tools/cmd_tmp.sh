set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --config conformer > gpurun_out/bc.log 2>&1 || { tail -30 gpurun_out/bc.log; exit 1; }
tail -1 gpurun_out/bc.log
