"""Run bench.py's N4 steady-state leg alone (tuning / profiling): python tools/cfk_steady.py [uniform|zipf] [batches]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cassandra-accord_amd")]
import bench  # noqa: E402

dist = sys.argv[1] if len(sys.argv) > 1 else "uniform"
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 5
top = int(sys.argv[3]) if len(sys.argv) > 3 else 10
print(json.dumps({dist: bench.cfk_steady_leg(0, dist=dist, n_batches=nb, top_n=top)}), flush=True)
