set -e
bash tools/gpu_check.sh defer "deferred or step_matches or full_size or reduce_loss"
