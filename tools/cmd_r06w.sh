set -u
# GRU backward with step s-1's loads prefetched (tools/gru_probe.hip)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06w; mkdir -p $O
timeout -k 10 120 probe_bin/gru_probe > $O/gru_probe.txt 2>&1 || { tail $O/gru_probe.txt; exit 1; }
head -4 $O/gru_probe.txt
