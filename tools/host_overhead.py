"""Host-side cost per forward call (tiny problem, GPU time negligible): module path, ops.forward,
the bare C-ABI call, and a HIP-graph replay of the module call. Analysis tool."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama-fft_amd"))
import torch  # noqa: E402
from bcfft import _lib, ops  # noqa: E402
from patch_llama_fft import BlockCirculantLinear  # noqa: E402


def per_call(fn, iters=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / iters * 1e6


def main():
    k, m, b, n = 4096, 4096, 128, int(sys.argv[1]) if len(sys.argv) > 1 else 4
    layer = BlockCirculantLinear(k, m, block_size=b, bias=False).cuda().eval()
    x = torch.randn(n, k, device="cuda")
    with torch.inference_mode():
        spec = layer._spectra(layer.c)
        y = torch.empty(n, m, device="cuda")
        lib = _lib.load()
        stream = _lib.stream_handle(x.device)
        args = (x.data_ptr(), _lib.dtype_code(x.dtype), n, k, m, b, spec.data_ptr(), 0, _lib.BCFFT_NONE,
                y.data_ptr(), _lib.dtype_code(y.dtype), _lib.ALGOS["auto"], stream)
        print(f"N={n}: module call      {per_call(lambda: layer(x)):7.1f} us/call (host issue rate)")
        print(f"N={n}: ops.forward      {per_call(lambda: ops.forward(x, spec, None, b, m)):7.1f} us/call")
        print(f"N={n}: C-ABI call       {per_call(lambda: lib.bcfft_forward_algo(*args)):7.1f} us/call")
        print(f"N={n}: stream_handle    {per_call(lambda: _lib.stream_handle(x.device)):7.1f} us/call")
        print(f"N={n}: torch.empty      {per_call(lambda: torch.empty(n, m, device='cuda')):7.1f} us/call")
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            layer(x)
            with torch.cuda.graph(g, stream=s):
                yg = layer(x)
        torch.cuda.current_stream().wait_stream(s)
        print(f"N={n}: graph replay     {per_call(lambda: g.replay()):7.1f} us/call")
        ref = layer(x)
        g.replay()
        torch.cuda.synchronize()
        print("graph output matches eager:", bool(torch.equal(yg, ref)))


if __name__ == "__main__":
    main()
