set -u
# HEAD check after the second session restart: the round-end rehearsal (pytest -m gpu, smoke, default
# bench line), then one replayed step of each bench config kernel by kernel
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/cmd_rehearsal.sh r05ad || exit 1
bash tools/cmd_step_breakdown.sh r05ad_sb
