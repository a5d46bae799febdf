"""Ablation (results invalid): the bf16 step with parts of the work removed, to price them.
ABL=grads  -> no LoRA dA/dB products (the side stream's work)
ABL=skinny -> LoRA down / g products replaced by nothing (u, g stay as they are)
ABL=nogdb  -> (valid) g and dB as separate streams over dy, dB on the side stream (the pre-fusion step)
python tools/ablate_side.py --steps 10 --warmup 3 --no-cpu-baseline"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ospo_amd import engine  # noqa: E402
import bench  # noqa: E402

abl = os.environ.get("ABL", "grads")
if abl == "grads":
    engine.SimPOEngine._lora_grads = lambda self, *a, **k: None
elif abl == "nogdb":  # valid results: g and dB as two streams over dy (dB on the side stream)
    engine.SimPOEngine._lora_g_db = lambda self, dy, g, Bcat, BT, M, par, u, gbase: (
        self._lora_g(dy, g, Bcat, BT, M, par), False)
elif abl == "skinny":
    engine.SimPOEngine._lora_down = lambda self, *a, **k: None
    engine.SimPOEngine._lora_g = lambda self, dy, g, Bcat, BT, M, par=0: self.gsc2[g.name][par]
bench.main()
