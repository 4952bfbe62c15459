set -u
# round-end state check (HEAD): the round-end rehearsal (pytest -m gpu, smoke, default
# bench line), then one replayed step of each bench config kernel by kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/cmd_rehearsal.sh r05ay || exit 1
bash tools/cmd_step_breakdown.sh r05ay_sb
