bench.py --mode agg --threads 20 --steps 10 --agg-op readat --level shrink --algo chacha20poly1305
