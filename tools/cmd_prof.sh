set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/round_profile.sh r01e > gpurun_out/r01e_profile.out 2>&1 || { tail -20 gpurun_out/r01e_profile.out; exit 1; }
tail -3 gpurun_out/r01e_profile.out
python tools/timeline.py gpurun_out/r01e/prof adam 1 > gpurun_out/r01e/timeline.txt 2>&1 || true
head -40 gpurun_out/r01e/timeline.txt
