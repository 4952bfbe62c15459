cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03s; mkdir -p $O
for V in "B2P_GEMM16_K64=0" "B2P_GEMM16_K64=1" "B2P_GEMM16_GROUP=4"; do
  env $V timeout -k 10 120 python -u tools/gemm_ab.py > $O/ab_$V.txt 2>&1 || { r=$?; echo "ab rc=$r"; exit $r; }
  echo "== $V"; grep -v amdgpu $O/ab_$V.txt | grep -v build_lib
done
