set -e
bash tools/gpu_check.sh epi16 "gemm or gru or encoder_layer or step_matches or full_size or reduce_loss or attention"
