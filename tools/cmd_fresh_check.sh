set -u
# Round-end rehearsal from a tracked-files-only state: drop the locally built library and objects,
# then run exactly what the driver runs (pytest -m gpu, smoke(), bench.py --gpus 1); each entry
# point builds the library itself.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-fresh}
mkdir -p $O
rm -rf build wav2vec2forbrain_amd/libb2p_hip.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
T0=$SECONDS
timeout -k 10 900 python bench.py --gpus 1 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json; echo "bench wall $((SECONDS - T0)) s" | tee $O/bench_wall.txt
# the same Trainer steps without graph replay (eager issue from Python), for the eager-vs-replayed line
timeout -k 10 600 python bench.py --graph 0 --no-cpu-baseline --no-parity > $O/bench_eager.json 2> $O/bench_eager.err || { tail -20 $O/bench_eager.err; exit 1; }
tail -1 $O/bench_eager.json
