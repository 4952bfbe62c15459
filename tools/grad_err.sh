set -e
timeout -k 5 200 python tools/loss_err.py 32 1024
timeout -k 5 100 python tools/loss_err.py 2 512
timeout -k 5 100 python tools/loss_err.py 8 512
