set -e
timeout -k 5 120 python tools/attn_bench.py
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "attention" 2>&1 | tail -3
