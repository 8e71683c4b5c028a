"""Debug: bench.py with the channel-padded thin-conv paths off (engine._PAD_THIN_CONVS)."""
import os, runpy, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from adaptsegnet_amd import engine
engine._PAD_THIN_CONVS = False
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path("bench.py", run_name="__main__")
