"""Do kernels on two HIP streams run concurrently on MI355X? Times a chain of GEMMs on one stream
alone, a side workload alone, and both launched together (no dependencies), eager and in a graph.
Side workloads: a spin kernel (torch.cuda._sleep) and a chain of small copies."""
import json

import torch


def main():
    dev = torch.device("cuda", 0)
    a = torch.randn(2048, 4096, device=dev, dtype=torch.bfloat16)
    b = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    src = torch.randn(1 << 22, device=dev)
    dst = torch.empty_like(src)
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream(priority=-1)
    side_lo = torch.cuda.Stream()

    def mm_chain():
        for _ in range(40):
            torch.mm(a, b)

    def spin():
        torch.cuda._sleep(2_000_000)

    def copies():
        for _ in range(200):
            dst.copy_(src)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t.record()
        fn()
        t1.record()
        torch.cuda.synchronize()
        return round(t.elapsed_time(t1) * 1e3, 1)

    res = {"mm_alone_us": timed(mm_chain), "spin_alone_us": timed(spin), "copies_alone_us": timed(copies)}
    for nm, sfn in (("spin", spin), ("copies", copies)):
        for sname, st in (("hiprio", side), ("normal", side_lo)):
            def both():
                st.wait_stream(main_s)
                with torch.cuda.stream(st):
                    sfn()
                mm_chain()
                main_s.wait_stream(st)
            res[f"mm+{nm}_{sname}_us"] = timed(both)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
