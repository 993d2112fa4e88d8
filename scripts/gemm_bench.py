"""Micro-benchmark of the update's GEMM shapes through lrl_gemm_f32 (development tool).
usage: python scripts/gemm_bench.py [path/to/liblrl.so ...]"""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = int(os.environ.get("GEMM_BENCH_B", "24576"))  # 4096: the rollout act's row count
dev = "cuda:0"
# (name, layout, epi, M, N, K, groups-as-separate-calls)
SHAPES = [
    ("AC2 fwd  NT 512->256 x2", 0, 2, B, 256, 512),
    ("AC1 fwd  NT 60->1024", 0, 2, B, 1024, 60),
    ("AC1 fwd  NT 64->1024 (padded X)", 0, 2, B, 1024, 64),
    ("D1 fwd   NT 630->256 gather", 0, 2, B, 256, 630),
    ("E1 fwd   NT 18->256 gather", 0, 2, B, 256, 18),
    ("E1 noelu NT 18->256 gather", 0, 1, B, 256, 18),
    ("E1 plain NT 18->256", 0, 1, B, 256, 18),
    ("E1 k16   NT 16->256", 0, 1, B, 256, 16),
    ("E2 fwd   NT 256->128", 0, 2, B, 128, 256),
    ("E2 noelu NT 256->128", 0, 1, B, 128, 256),
    ("E3 fwd   NT 128->18", 0, 1, B, 18, 128),
    ("D2 fwd   NT 256->32", 0, 2, B, 32, 256),
    ("dH1      NN 256->512 x2", 2, 3, B, 512, 256),
    ("dLat     NN 1024->18", 2, 0, B, 18, 1024),
    ("dHe2     NN 18->128", 2, 3, B, 128, 18),
    ("dHD1     NN 32->256", 2, 3, B, 256, 32),
    ("dW2      TN 256x512", 3, 4, 256, 512, B),
    ("dWD1     TN 256x630 gather", 3, 4, 256, 630, B),
    ("dWe1     TN 256x18 gather", 3, 4, 256, 18, B),
    ("dWe3     TN 18x128", 3, 4, 18, 128, B),
    ("dW1      TN 1024x60", 3, 4, 1024, 60, B),
    ("dWD2     TN 32x256", 3, 4, 32, 256, B),
    ("long-K   NT 4096->256", 0, 2, B, 256, 4096),
]
if os.environ.get("GEMM_BENCH_FILTER"):
    SHAPES = [s for s in SHAPES if os.environ["GEMM_BENCH_FILTER"] in s[0]]


def run(libpath):
    L = C.CDLL(libpath)
    L.lrl_gemm_f32.restype = C.c_int32
    p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    out = []
    for name, lay, epi, M, N, K in SHAPES:
        gather = "gather" in name
        if lay == 0:
            src = torch.randn(B + 100 if gather else M, K, device=dev)
            A, lda = src, K
            W = torch.randn(N, K, device=dev)
            Bm, ldb = W, K
            rows = torch.randperm(B + 100, device=dev)[:M].contiguous() if gather else None
        elif lay == 2:
            A, lda = torch.randn(M, K, device=dev), K
            Bm, ldb = torch.randn(K, N, device=dev), N
            rows = None
        else:
            A, lda = torch.randn(K, M, device=dev), M
            Bm, ldb = torch.randn(K + 100 if gather else K, N, device=dev), N
            rows = torch.randperm(K + 100, device=dev)[:K].contiguous() if gather else None
        Cm = torch.empty(M, N, device=dev)
        bias = torch.randn(N if lay != 3 else M, device=dev)
        aux = torch.randn(M, N, device=dev) if epi == 3 else None
        ws = torch.empty(128 * (M * N + M), device=dev) if lay == 3 else None

        def call():
            cs = C.c_void_p(torch.cuda.current_stream().cuda_stream)  # (the capture stream under GEMM_BENCH_GRAPH)
            rc = L.lrl_gemm_f32(lay, epi, M, N, K, p(A), C.c_int64(lda), p(Bm), C.c_int64(ldb), p(Cm),
                                C.c_int64(N), p(bias), p(aux), C.c_int64(N), p(rows), p(ws),
                                C.c_int64(ws.numel() if ws is not None else 0), cs)
            assert rc == 0, rc
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        if os.environ.get("GEMM_BENCH_GRAPH"):  # the n launches captured once as a HIP graph, replayed
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(n):
                    call()
            g.replay()
            torch.cuda.synchronize()
            e0.record()
            g.replay()
            e1.record()
        else:
            e0.record()
            for _ in range(n):
                call()
            e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
        out.append((name, us, tf))
    return out


if __name__ == "__main__":
    libs = sys.argv[1:] or [os.path.join(ROOT, "rapid-locomotion-rl_amd", "csrc", "liblrl.so")]
    # warm the clocks, then alternate the libraries twice and keep each one's best time per shape
    run(libs[0])
    res = {}
    for _ in range(2):
        for lib in libs:
            r = run(lib)
            res[lib] = r if lib not in res else [min(x, y, key=lambda z: z[1]) for x, y in zip(res[lib], r)]
    for i, (name, *_r) in enumerate(SHAPES):
        print(f"{name:32s}" + "".join(f"  {res[l][i][1]:8.1f}us {res[l][i][2]:6.1f}TF" for l in libs))
