"""A/B of where a layer's LoRA dA work joins the side stream (SimPOEngine(side_after_norm=...)):
SIDE_AFTER_NORM=1 enqueues it after the layer's input-norm backward (the default since round 3),
SIDE_AFTER_NORM=0 right after its q|k|v dX GEMM.
python tools/side_order_ab.py --no-cpu-baseline   (bench.py's flags; one JSON line)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import engine  # noqa: E402
import bench  # noqa: E402

if "SIDE_AFTER_NORM" in os.environ:
    _init = engine.SimPOEngine.__init__

    def _patched(self, *a, **k):
        k.setdefault("side_after_norm", os.environ["SIDE_AFTER_NORM"] == "1")
        _init(self, *a, **k)

    engine.SimPOEngine.__init__ = _patched
bench.main()
