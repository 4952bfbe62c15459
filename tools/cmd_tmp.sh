set -e
bash tools/gpu_check.sh ctc3 "ctc or colsum or step_matches or full_size or reduce_loss or front_end or layernorm or conformer or gemm"
