JFSX_EVENT_SPIN=1 (reverted knob) bench.py --mode agg --threads 20 --steps 10 --no-cpu --agg-op seal --agg-max-mb 16
