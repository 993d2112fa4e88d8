"""x6d (LDS-DMA forward / backward-data) against gemm_x6_kernel on the update's and the act's batch-major shapes
(development tool): bit-identity and time through lrl_gemm_f32, lrl_debug_gemm_paths(4) = x6d off.
usage: python scripts/x6d_bench.py"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dev = "cuda:0"
SHAPES = [  # (name, layout, epi, M, N, K, gather)
    ("AC2 fwd NT 512->256", 0, 2, 24576, 256, 512, False),
    ("AC1 fwd NT 64->1024", 0, 2, 24576, 1024, 64, False),
    ("AC3 fwd NT 256->128", 0, 2, 24576, 128, 256, False),
    ("D1 fwd NT 640->256 gather", 0, 2, 24576, 256, 640, True),
    ("dH1 NN 256->512", 2, 3, 24576, 512, 256, False),
    ("dH2 NN 128->256", 2, 3, 24576, 256, 128, False),
    ("dHD1 NN 32->256", 2, 3, 24576, 256, 32, False),
    ("act AC2 NT 512->256", 0, 2, 4096, 256, 512, False),
    ("act AC1 NT 64->1024", 0, 2, 4096, 1024, 64, False),
]


def main():
    L = C.CDLL(os.environ.get("LRL_LIB", os.path.join(ROOT, "rapid-locomotion-rl_amd/csrc/liblrl.so")))
    L.lrl_gemm_f32.restype = C.c_int32
    L.lrl_debug_gemm_paths.restype = C.c_int32
    p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None
    torch.manual_seed(0)
    ok = True
    for name, lay, epi, M, N, K, gather in SHAPES:
        src = torch.randn(M + 100 if gather else M, K, device=dev)
        rows = torch.randperm(M + 100, device=dev)[:M].contiguous() if gather else None
        W, ldb = (torch.randn(N, K, device=dev), K) if lay == 0 else (torch.randn(K, N, device=dev), N)
        bias = torch.randn(N, device=dev)
        aux = torch.randn(M, N, device=dev) if epi == 3 else None

        def call(mask, out):
            L.lrl_debug_gemm_paths(mask)
            st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
            rc = L.lrl_gemm_f32(lay, epi, M, N, K, p(src), C.c_int64(K), p(W), C.c_int64(ldb), p(out), C.c_int64(N),
                                p(bias), p(aux), C.c_int64(N), p(rows), None, C.c_int64(0), st)
            assert rc == 0

        t, outs = {}, {}
        for mask in (4, 8, 4, 8):
            out = torch.empty(M, N, device=dev)
            for _ in range(3):
                call(mask, out)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                call(mask, out)
            e1.record()
            torch.cuda.synchronize()
            t.setdefault(mask, []).append(e0.elapsed_time(e1) / 20 * 1e3)
            outs[mask] = out
        same = torch.equal(outs[4], outs[8])
        ok = ok and same
        x6, x6d = min(t[4]), min(t[8])
        print(json.dumps({"shape": name, "bit_identical": same, "x6_us": round(x6, 2), "x6d_us": round(x6d, 2),
                          "speedup": round(x6 / x6d, 3), "x6d_tflops": round(2.0 * M * N * K / (x6d * 1e-6) / 1e12, 1)}),
              flush=True)
    L.lrl_debug_gemm_paths(0)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
