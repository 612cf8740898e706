"""C1 leg alone (B=1, N=20 controller step through Nmpc), for a kernel trace of its launch structure."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
print(json.dumps(bench.bench_c1(0, True, steps=int(os.environ.get("STEPS", 100)))))
