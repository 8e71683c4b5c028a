"""Debug: run a script (or pytest) against an alternative build of libadaptseg.so.
   python tools/dbg/with_lib.py LIB.so script.py args...   |   ... LIB.so -m pytest args..."""
import os, runpy, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import adaptsegnet_amd._lib as L
L.LIB_PATH = os.path.abspath(sys.argv[1])
print("libadaptseg:", L.LIB_PATH, flush=True)
if sys.argv[2] == "-m":
    sys.argv = [sys.argv[3]] + sys.argv[4:]
    runpy.run_module(sys.argv[0], run_name="__main__")
else:
    sys.argv = sys.argv[2:]
    runpy.run_path(sys.argv[0], run_name="__main__")
