"""x6t (LDS-DMA weight gradient) against gemm_x6_kernel on the update's weight-gradient shapes (development tool):
bit-identity and time through lrl_gemm_f32 (split-k partials + seg_reduce), lrl_debug_gemm_paths(2) = x6t off.
usage: python scripts/x6t_bench.py"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = int(os.environ.get("GEMM_BENCH_B", "24576"))
dev = "cuda:0"
SHAPES = [("dW2 TN 256x512", 256, 512, 512), ("dW3 TN 128x256", 128, 256, 256), ("dWe2 TN 128x256", 128, 256, 256),
          ("dW1 TN 1024x60", 1024, 60, 64)]


def main():
    L = C.CDLL(os.environ.get("LRL_LIB", os.path.join(ROOT, "rapid-locomotion-rl_amd/csrc/liblrl.so")))
    L.lrl_gemm_f32.restype = C.c_int32
    L.lrl_debug_gemm_paths.restype = C.c_int32
    p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None
    torch.manual_seed(0)
    ok = True
    for name, M, N, ldx in SHAPES:
        K = B
        dY, X = torch.randn(K, M, device=dev), torch.randn(K, ldx, device=dev)
        ws = torch.empty(256 * (M * N + M), device=dev)
        outs = {}

        def call(mask, out, db):
            L.lrl_debug_gemm_paths(mask)
            st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
            rc = L.lrl_gemm_f32(3, 4, M, N, K, p(dY), C.c_int64(M), p(X), C.c_int64(ldx), p(out), C.c_int64(N), p(db),
                                None, C.c_int64(0), None, p(ws), C.c_int64(ws.numel()), st)
            assert rc == 0

        t = {}
        for mask in (2, 0, 2, 0):
            out, db = torch.empty(M, N, device=dev), torch.empty(M, device=dev)
            for _ in range(3):
                call(mask, out, db)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                call(mask, out, db)
            e1.record()
            torch.cuda.synchronize()
            t.setdefault(mask, []).append(e0.elapsed_time(e1) / 20 * 1e3)
            outs[mask] = (out, db)
        same = torch.equal(outs[2][0], outs[0][0]) and torch.equal(outs[2][1], outs[0][1])
        ok = ok and same
        rec = {"shape": name, "bit_identical": same, "x6_us": round(min(t[2]), 2), "x6t_us": round(min(t[0]), 2),
               "speedup": round(min(t[2]) / min(t[0]), 3)}
        print(json.dumps(rec), flush=True)
    L.lrl_debug_gemm_paths(0)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
