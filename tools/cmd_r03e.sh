cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 300 python -u tools/fixture_err.py conformer_large_b2 large960_bs32 conformer_large_ft_bs8 > $O/fixture_err.txt 2>&1; echo "fixture_err rc=$?"
grep -E "fp32\[-\]|fp32\[attn\]|all-fp32" $O/fixture_err.txt
timeout -k 10 300 python -u tools/ld_adam_probe.py tiny_a > $O/ld_probe.txt 2>&1; echo "ld_probe rc=$?"; tail -20 $O/ld_probe.txt
timeout -k 10 700 python -u tools/trainer_capture_probe.py > $O/probe.txt 2>&1; echo "probe rc=$?"
grep -vE "^\s*$" $O/probe.txt | tail -40
