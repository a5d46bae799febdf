"""A/B for config 5: the MXFP8 copies of the attention output / dqkv written by the attention kernels
(default) vs the standalone quantizer (--old: ops.flash_attn_* drop mx and quant_mx8 runs after them,
which is what the engine did before).  Runs bench.py's step in-process; prints its JSON line."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
old = "--old" in sys.argv
if old:
    sys.argv.remove("--old")
    from ospo_amd import ops
    _fwd, _bwd = ops.flash_attn_fwd, ops.flash_attn_bwd

    def fwd(*a, mx=None, **k):
        r = _fwd(*a, **k)
        if mx is not None:
            ops.quant_mx8(a[4][: a[6] * a[7]], mx)
        return r

    def bwd(*a, mx=None, **k):
        r = _bwd(*a, **k)
        if mx is not None:
            ops.quant_mx8(a[9][: a[10] * a[11]], mx)
        return r

    ops.flash_attn_fwd, ops.flash_attn_bwd = fwd, bwd
import bench  # noqa: E402

bench.main()
