set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05z; mkdir -p $O
timeout -k 10 300 python3 tools/blaslt_count.py base > $O/count_base.txt 2>&1 || { tail -20 $O/count_base.txt; exit 1; }
cat $O/count_base.txt | grep -v amdgpu.ids
