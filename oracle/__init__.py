"""CPU oracle for the IR->RGB GAN train step -- TEST INFRASTRUCTURE ONLY.

This package is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (the HIP kernels behind ``include/irgan.h``) never calls into
here and fails loudly when its extension is missing.

``oracle.step`` is an fp32 PyTorch-CPU restatement of the reference's hot path
(``/root/reference/Code/ir_colorization.py``, cited as ``ir:LINE``) written from
the math, not from the reference's source text.  It is pinned against golden
vectors produced by executing the reference itself in the build container
(``tests/golden/make_golden.py``; fixtures in ``tests/golden/*.npz``).
"""
from .step import *  # noqa: F401,F403
