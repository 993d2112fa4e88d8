"""Split-count sweep of the update's weight-gradient (TN, split-k + fixed-order reduce) shapes through
lrl_gemm_f32 (development tool; LRL_GEMM_SPLITS overrides gemm_pick_splits in that entry point only).
usage: python scripts/tn_sweep.py"""
import ctypes as C
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = 24576
dev = "cuda:0"
SHAPES = [("dW2 256x1024", 256, 1024, False, 0), ("dW3 256x256", 256, 256, False, 0),
          ("dW1 1024x60", 1024, 60, False, 64), ("dWD1 256x630 g", 256, 630, True, 640),
          ("dWe2 128x256", 128, 256, False, 0), ("dWe1 256x18 g", 256, 18, True, 0), ("dWe3 18x128", 18, 128, False, 0),
          ("dWD2 32x256", 32, 256, False, 0), ("dWD3 18x32", 18, 32, False, 0)]
SPLITS = [0, 8, 16, 32, 64, 128, 256]


def main():
    L = C.CDLL(os.path.join(ROOT, "rapid-locomotion-rl_amd", "csrc", "liblrl.so"))
    L.lrl_gemm_f32.restype = C.c_int32
    p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    torch.randn(8192, 8192, device=dev) @ torch.randn(8192, 8192, device=dev)  # clocks
    for name, M, N, gather, ldb in SHAPES:
        K = B
        ldb = ldb or N
        A = torch.randn(K, M, device=dev)
        Bm = torch.randn(K + 100 if gather else K, ldb, device=dev)
        rows = torch.randperm(K + 100, device=dev)[:K].contiguous() if gather else None
        Cm = torch.empty(M, N, device=dev)
        db = torch.empty(M, device=dev)
        ws = torch.empty(256 * (M * N + M), device=dev)
        line = []
        for s in SPLITS:
            os.environ["LRL_GEMM_SPLITS"] = str(s)

            def call():
                rc = L.lrl_gemm_f32(3, 4, M, N, K, p(A), C.c_int64(M), p(Bm), C.c_int64(ldb), p(Cm), C.c_int64(N),
                                    p(db), None, C.c_int64(0), p(rows), p(ws), C.c_int64(ws.numel()), st)
                assert rc == 0, rc
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    call()
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / 10 * 1e3)
            line.append(f"{'auto' if s == 0 else s}:{best:6.1f}")
        print(f"{name:16s} " + "  ".join(line), flush=True)


if __name__ == "__main__":
    main()
