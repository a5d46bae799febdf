"""What an event costs the stream it is recorded on / waited on (the engine's backward records one event per
adapter group on the main stream and waits on the side stream's events): N back-to-back writes of a
16 MiB buffer on the main stream, plain vs with an event recorded after each, vs with a wait on an already
completed side-stream event before each, vs both.  Prints per-launch microseconds (CUDA-event timed)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

N = 200


def main():
    dev = torch.device("cuda")
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev, priority=-1)
    buf = torch.zeros(4 << 20, device=dev)  # 16 MiB: every launch leaves dirty lines in L2
    done = torch.cuda.Event()
    with torch.cuda.stream(side):
        torch.zeros(1, device=dev).add_(1)
    done.record(side)
    torch.cuda.synchronize()

    def run(mode):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        evs = [torch.cuda.Event() for _ in range(N)]
        e0.record(main_s)
        for i in range(N):
            if mode in ("wait", "both"):
                main_s.wait_event(done)
            buf.add_(1.0)
            if mode in ("record", "both"):
                evs[i].record(main_s)
        e1.record(main_s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / N

    res = {}
    for rep in range(3):
        for mode in ("plain", "record", "wait", "both"):
            res.setdefault(mode, []).append(run(mode))
    print(json.dumps({k: round(sorted(v)[1], 2) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
