bench.py --algo chacha20poly1305 --steps 10 --warmup 2
