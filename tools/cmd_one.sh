set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/one; mkdir -p $O
timeout -k 10 300 python -u -m pytest ${2:-tests} -m "${3:-gpu}" -x -v --timeout 120 --timeout-method thread -k "$1" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
