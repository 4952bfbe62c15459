set -e
timeout -k 5 60 python tools/gru_bench.py
timeout -k 5 60 python tools/gru_bench.py 32 249 128
