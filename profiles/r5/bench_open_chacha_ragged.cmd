bench.py --algo chacha20poly1305 --mode open --ragged --steps 10 --warmup 2
