bench.py 
