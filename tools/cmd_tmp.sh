set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/g512 -o run -- python3 -u tools/gru512_bench.py > gpurun_out/g512.log 2>&1 || { tail -20 gpurun_out/g512.log; exit 1; }
grep "gru H" gpurun_out/g512.log
python tools/prof_summary.py gpurun_out/g512 4 12 2>&1 | cut -c1-160
