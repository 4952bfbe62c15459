set -u
# GRU forward recurrence ablations and the split-order step (tools/gru_probe.hip)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 120 probe_bin/gru_probe > $O/gru_probe2.txt 2>&1 || { tail $O/gru_probe2.txt; exit 1; }
cat $O/gru_probe2.txt
