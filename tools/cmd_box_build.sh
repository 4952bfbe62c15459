set -u
# The library built from source ON the GPU box (the snapshot's .so, its stamp and objects removed first),
# then the kernel-level GPU tests, smoke() and a base bench line on that build. usage: bash tools/cmd_box_build.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-box_build}; mkdir -p $O
sha256sum wav2vec2forbrain_amd/libb2p_hip.so > $O/shipped_sha.txt
rm -rf build wav2vec2forbrain_amd/libb2p_hip.so wav2vec2forbrain_amd/libb2p_hip.so.sha
(while sleep 45; do echo "building $(date +%T)"; done) & HB=$!
T0=$SECONDS
timeout -k 10 900 python3 -m wav2vec2forbrain_amd.build_lib -v > $O/build.log 2>&1; rc=$?
kill $HB
echo "box build rc=$rc wall $((SECONDS - T0)) s" | tee $O/build_wall.txt
[ $rc -ne 0 ] && { tail -30 $O/build.log; exit $rc; }
sha256sum wav2vec2forbrain_amd/libb2p_hip.so > $O/box_sha.txt; cat wav2vec2forbrain_amd/libb2p_hip.so.sha >> $O/box_sha.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-conformer --no-extra > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('base', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['max_rel_err'])"
