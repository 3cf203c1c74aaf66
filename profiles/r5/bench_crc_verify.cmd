bench.py --mode crc --steps 10 --warmup 2
