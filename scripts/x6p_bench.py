"""x6p (pre-split weight planes, LDS-DMA) against gemm_x6_kernel on the update's weight products (development tool).
Checks the two are bit-identical and times both through lrl_gemm_f32 (layout | 0x100 = planes path; the planes are
built inside the timed call, as the update builds them once per optimiser step for several products).
usage: python scripts/x6p_bench.py"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = int(os.environ.get("GEMM_BENCH_B", "24576"))
dev = "cuda:0"
SHAPES = [  # (name, layout, epi, N, K, gather)
    ("AC2 fwd NT 512->256", 0, 2, 256, 512, False),
    ("AC1 fwd NT 64->1024", 0, 2, 1024, 64, False),
    ("AC3 fwd NT 256->128", 0, 2, 128, 256, False),
    ("E2 fwd NT 256->128", 0, 2, 128, 256, False),
    ("D1 fwd NT 640->256 gather", 0, 2, 256, 640, True),
    ("dH1 NN 256->512", 2, 3, 512, 256, False),
    ("dH2 NN 128->256", 2, 3, 256, 128, False),
    ("dHD1 NN 32->256", 2, 3, 256, 32, False),
    ("plain NT 512->256", 0, 0, 256, 512, False),
]


def main():
    L = C.CDLL(os.environ.get("LRL_LIB", os.path.join(ROOT, "rapid-locomotion-rl_amd/csrc/liblrl.so")))
    L.lrl_gemm_f32.restype = C.c_int32
    L.lrl_last_error.restype = C.c_char_p
    p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None
    torch.manual_seed(0)
    out = []
    for name, lay, epi, N, K, gather in SHAPES:
        M = B
        src = torch.randn(B + 100 if gather else M, K, device=dev)
        rows = torch.randperm(B + 100, device=dev)[:M].contiguous() if gather else None
        if lay == 0:
            W, ldb = torch.randn(N, K, device=dev), K
        else:
            W, ldb = torch.randn(K, N, device=dev), N
        bias = torch.randn(N, device=dev)
        aux = torch.randn(M, N, device=dev) if epi == 3 else None
        ws = torch.empty(3 * N * ((K + 15) // 16 * 16), device=dev)
        C0 = torch.empty(M, N, device=dev)
        C1 = torch.empty(M, N, device=dev)

        def call(planes, Cm):
            st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
            rc = L.lrl_gemm_f32(lay | (0x100 if planes else 0), epi, M, N, K, p(src), C.c_int64(K), p(W),
                                C.c_int64(ldb), p(Cm), C.c_int64(N), p(bias), p(aux), C.c_int64(N), p(rows), p(ws),
                                C.c_int64(ws.numel()), st)
            if rc != 0:
                raise RuntimeError(f"{name}: {L.lrl_last_error().decode()}")

        call(False, C0)
        call(True, C1)
        torch.cuda.synchronize()
        same = bool(torch.equal(C0, C1))
        ref = (src[rows] if gather else src).double() @ (W.double().t() if lay == 0 else W.double())
        err = float(((C1.double() - (ref if epi == 0 else C1.double() * 0 + C1.double())).abs().max()) if epi == 0 else 0.0)
        t = {}
        for planes, Cm in ((False, C0), (True, C1), (False, C0), (True, C1)):
            for _ in range(3):
                call(planes, Cm)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                call(planes, Cm)
            e1.record()
            torch.cuda.synchronize()
            t.setdefault(planes, []).append(e0.elapsed_time(e1) / 20 * 1e3)
        x6, x6p = min(t[False]), min(t[True])
        tf = 2.0 * M * N * K / (x6p * 1e-6) / 1e12
        rec = {"shape": name, "bit_identical": same, "x6_us": round(x6, 2), "x6p_us": round(x6p, 2),
               "speedup": round(x6 / x6p, 3), "x6p_tflops": round(tf, 1)}
        if epi == 0:
            rec["max_abs_err_vs_fp64"] = err
        out.append(rec)
        print(json.dumps(rec), flush=True)
    return 0 if all(r["bit_identical"] for r in out) else 1


if __name__ == "__main__":
    sys.exit(main())
