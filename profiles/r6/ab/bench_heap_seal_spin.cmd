JFSX_EVENT_SPIN=1 (reverted knob) bench.py --mode agg --threads 20 --steps 10 --no-cpu --buffers heap --agg-op seal --agg-crc seg
