set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "attention or encoder_layer or step_matches or full_size or step_graph" > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/tr_attn -o run -- python -u tools/attn_bench.py > gpurun_out/attn.log 2>&1 || { tail -30 gpurun_out/attn.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -30 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['ctc_loss'])"
