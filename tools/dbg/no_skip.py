"""Debug A/B: run a script with engine.bf16_only forced False (every BN pass writes its fp32
output too, as before the bf16-only skipping).  python tools/dbg/no_skip.py script.py args..."""
import os, runpy, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from adaptsegnet_amd import engine
engine.bf16_only = lambda *a, **kw: False
sys.argv = sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
