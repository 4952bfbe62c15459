set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/gelu; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python tools/epi_bench.py 7968 3072 768 > $O/epi.jsonl 2> $O/epi.err || { tail -5 $O/epi.err; exit 1; }
cat $O/epi.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
tail -1 $O/b.json | cut -c1-220
