set -u
# full GPU suite + the default bench line + eager-vs-replay step times: bash tools/cmd_full.sh <tag> [pytest -k expr]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-full}
mkdir -p $O
K=${2:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|rel \[|worst relative" $O/pytest.log | tail -30
tail -3 $O/pytest.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1; rc2=$?
tail -c 1500 $O/bench.log
[ $rc2 -ne 0 ] && exit $rc2
timeout -k 10 300 python -u bench.py --graph 0 --no-cpu-baseline --no-parity --no-roofline > $O/bench_eager.log 2>&1; rc3=$?
grep -o '"ms_per_step": [0-9.]*' $O/bench_eager.log
exit $rc3
