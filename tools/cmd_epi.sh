set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/epi; mkdir -p $O
timeout -k 10 120 python tools/epi_bench.py 7968 3072 768 > $O/base.jsonl 2> $O/base.err || { tail -5 $O/base.err; exit 1; }
cat $O/base.jsonl
timeout -k 10 120 python tools/epi_bench.py 7968 4096 1024 > $O/conf.jsonl 2> $O/conf.err || { tail -5 $O/conf.err; exit 1; }
cat $O/conf.jsonl
