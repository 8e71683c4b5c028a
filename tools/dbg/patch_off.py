"""Debug A/B: run a script with one engine predicate forced False, e.g. ``bf16_only`` (every BN
pass writes its fp32 output too) or ``_copy_pays`` (no epilogue-written bf16 operand copies).
    python tools/dbg/patch_off.py NAME script.py args..."""
import os, runpy, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from adaptsegnet_amd import engine
setattr(engine, sys.argv[1], lambda *a, **kw: False)
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
