"""bench.py with the engine's F32X3 operand copies switched off (--no-x3-copies): the Bottleneck
convs then read fp32 operands on the register-staged kernel (conv_x3.hpp) — the A arm of the
term-image A/B (experiments/ab_copies.sh).  Not product code."""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from adaptsegnet_amd import engine  # noqa: E402

if "--no-x3-copies" in sys.argv:
    sys.argv.remove("--no-x3-copies")
    engine.bf16_operands = engine.lowp_storage
sys.argv[0] = os.path.join(REPO, "bench.py")
runpy.run_path(sys.argv[0], run_name="__main__")
