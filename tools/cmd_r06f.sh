set -u
# epilogue ablation of the fused FFN GEMMs (base and Conformer shapes) and the N = 768 / 1024 shapes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06f; mkdir -p $O
for s in "7968 3072 768" "7968 768 3072" "7968 4096 1024"; do
  timeout -k 10 120 python3 -u tools/epi_ab.py $s >> $O/epi_ab.txt 2>&1 || { tail -5 $O/epi_ab.txt; exit 1; }
done
grep -v amdgpu $O/epi_ab.txt
