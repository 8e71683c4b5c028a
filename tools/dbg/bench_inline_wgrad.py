"""Debug: bench.py with the weight-gradient GEMMs on the main stream (no side stream)."""
import os, runpy, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from adaptsegnet_amd import engine
engine.WgradStream.launch = lambda self, fn, *tensors: fn()
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path("bench.py", run_name="__main__")
