"""How much do per-launch HIP event pairs add to a ~80 us kernel? Compares (a) an event pair
around every launch, (b) one pair around K back-to-back launches, (c) one pair around a HIP
graph of K launches. Run under rocprofv3 --kernel-trace --stats for the ground truth."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from patch_llama_fft import BlockCirculantLinear  # noqa: E402


def main():
    k = m = 4096
    b, n, steps = 128, 8192, 50
    torch.manual_seed(1)
    layer = BlockCirculantLinear(k, m, block_size=b, bias=False).cuda().eval()
    x = torch.randn(n, k, device="cuda")
    st = torch.cuda.current_stream()
    with torch.inference_mode():
        for _ in range(10):
            layer(x)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        torch.cuda.synchronize()
        for s, e in ev:
            s.record(st)
            layer(x)
            e.record(st)
        torch.cuda.synchronize()
        a = sum(s.elapsed_time(e) for s, e in ev) / steps * 1e3
        s0, e0 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record(st)
        for _ in range(steps):
            layer(x)
        e0.record(st)
        torch.cuda.synchronize()
        bb = s0.elapsed_time(e0) / steps * 1e3
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        cs.wait_stream(st)
        with torch.cuda.stream(cs):
            layer(x)
            with torch.cuda.graph(g, stream=cs):
                for _ in range(steps):
                    layer(x)
        st.wait_stream(cs)
        g.replay()
        torch.cuda.synchronize()
        s0.record(st)
        g.replay()
        e0.record(st)
        torch.cuda.synchronize()
        c = s0.elapsed_time(e0) / steps * 1e3
    print(f"per-launch event pairs {a:.1f} us | one pair over {steps} launches {bb:.1f} us/launch | "
          f"graph of {steps} {c:.1f} us/launch")


if __name__ == "__main__":
    main()
