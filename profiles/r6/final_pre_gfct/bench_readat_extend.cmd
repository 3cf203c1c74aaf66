bench.py --mode agg --threads 20 --steps 10 --agg-op readat --level extend --algo chacha20poly1305
