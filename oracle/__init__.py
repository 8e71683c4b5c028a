"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the AdaptSegNet adversarial step.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / the timed CPU baseline.  The product path
(``adaptsegnet_amd``) never imports it and has no CPU fallback.

Parity pinning: ``reference_torch`` restates the reference's arithmetic with stock
PyTorch CPU ops; it is pinned against golden vectors that ``tests/golden/gen_golden.py``
captured from the real reference modules (/root/reference/model/deeplab_multi.py,
model/discriminator.py, utils/loss.py) imported in the build container.
"""
