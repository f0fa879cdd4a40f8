"""Cost of cross-stream dependencies inside HIP graphs (the decode micro-batch overlap schedule).

Times N small kernels on the compute stream with k of them handing a tensor to a second stream
(event record / wait, the pattern DecoderLM._hidden_states_overlap uses for its all-reduces), both
captured in one HIP graph and eager. Prints one JSON line per variant.
"""
import json
import sys

import torch


def main():
    dev = torch.device("cuda", 0)
    x = torch.randn(1 << 20, device=dev)
    ys = [torch.randn(1 << 20, device=dev) for _ in range(2)]
    cur = torch.cuda.current_stream()
    side = torch.cuda.Stream(priority=-1)
    N = 256

    a = torch.randn(512, 4096, device=dev, dtype=torch.bfloat16)
    b = torch.randn(4096, 1536, device=dev, dtype=torch.bfloat16)
    state = {"main": "mul", "side": "add"}

    def main_op():
        if state["main"] == "mm":
            torch.mm(a, b)
        else:
            x.mul_(1.0001)

    def side_op(y):
        if state["side"] == "sleep":
            torch.cuda._sleep(int(state.get("cycles", 100)))
        else:
            y.add_(1.0)

    def body(cross: int, mode: str):
        evs = []
        for i in range(N):
            main_op()
            if cross and i % (N // cross) == 0:
                y = ys[i % 2]
                if mode == "wait_stream":
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        side_op(y)
                    cur.wait_stream(side)
                else:  # events, joined two kernels later (the overlap schedule)
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        side_op(y)
                        ev = torch.cuda.Event()
                        ev.record(side)
                    evs.append(ev)
                    if len(evs) > 1:
                        cur.wait_event(evs.pop(0))
        for ev in evs:
            cur.wait_event(ev)
        cur.wait_stream(side)

    def t_graph(cross, mode):
        body(cross, mode)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            body(cross, mode)
        g.replay()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            e.synchronize()
            best = min(best, s.elapsed_time(e) * 1e3)
        return best

    def t_eager(cross, mode):
        body(cross, mode)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        body(cross, mode)
        e.record()
        e.synchronize()
        return s.elapsed_time(e) * 1e3

    for main, sideop in (("mul", "add"), ("mul", "sleep"), ("mm", "add"), ("mm", "sleep")):
      state.update(main=main, side=sideop)
      for cross in (0, 64, 128):
        for mode in ("event", "wait_stream"):
            if cross == 0 and mode == "wait_stream":
                continue
            print(json.dumps({"main": main, "side": sideop, "kernels": N, "cross_stream_handoffs": cross, "mode": mode,
                              "graph_us": round(t_graph(cross, mode), 1), "eager_us": round(t_eager(cross, mode), 1)}),
                  flush=True)


if __name__ == "__main__":
    sys.exit(main())
