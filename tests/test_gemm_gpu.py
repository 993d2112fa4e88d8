"""fp32 MFMA GEMM of the native PPO update (csrc/lrl_gemm.hip, through lrl_gemm_f32) against a plain
torch fp32 reference of the same op: the three layouts an MLP's forward / backward-data / weight-gradient
need, every epilogue, gathered rows, ragged and unaligned shapes; the 64-aligned float4 shapes take the
LDS-DMA kernel, outputs <= 32 wide with k = 512 / 1024 the thin kernel (B in registers), the others the
register-staged one."""
import ctypes as C

import numpy as np
import pytest
import torch

from lrl import _abi

pytestmark = pytest.mark.gpu
dev = "cuda:0"


def _p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _gemm(layout, epi, M, N, K, A, lda, B, ldb, Cm, ldc, bias=None, aux=None, ld_aux=0, rows=None, ws=None):
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    nws = ws.numel() if ws is not None else 0
    _abi.check(_abi.lib().lrl_gemm_f32(C.c_int32(layout), C.c_int32(epi), C.c_int32(M), C.c_int32(N), C.c_int32(K),
                                       _p(A), C.c_int64(lda), _p(B), C.c_int64(ldb), _p(Cm), C.c_int64(ldc), _p(bias),
                                       _p(aux), C.c_int64(ld_aux), _p(rows), _p(ws), C.c_int64(nws), stream))
    torch.cuda.synchronize()


def _tol(ref, k):
    # fp32 accumulation-order difference: ~ sqrt(K) ulps of the magnitude of the products' sum
    return 2e-6 * np.sqrt(k) * (ref.abs().max().item() + 1.0)


@pytest.mark.parametrize("M,N,K,gather,epi", [(1024, 256, 512, True, 2), (2048, 1024, 64, False, 1),
                                               (1536, 128, 256, False, 0), (300, 200, 60, False, 2), (1000, 1024, 60, True, 2),
                                               (777, 256, 18, True, 2), (513, 18, 128, False, 1),
                                               (640, 256, 630, True, 2), (64, 64, 16, False, 0),
                                               (2048, 32, 512, True, 2), (4096, 18, 128, False, 1), (777, 7, 512, True, 0),
                                               (1000, 24, 1024, False, 1), (4096, 256, 18, True, 2), (300, 128, 30, False, 0)])
def test_forward_nt(M, N, K, gather, epi):
    g = torch.Generator(device=dev).manual_seed(M * 7 + N)
    src_rows = M + 37
    X = torch.randn(src_rows, K, device=dev, generator=g)
    W = torch.randn(N, K, device=dev, generator=g) / np.sqrt(K)
    b = torch.randn(N, device=dev, generator=g)
    rows = torch.randperm(src_rows, device=dev)[:M].contiguous() if gather else None
    Xm = X[rows] if gather else X[:M]
    ref = Xm @ W.T
    if epi >= 1:
        ref = ref + b
    if epi == 2:
        ref = torch.nn.functional.elu(ref)
    out = torch.full((M, N), float("nan"), device=dev)
    _gemm(0, epi, M, N, K, X, K, W, K, out, N, bias=b if epi else None, rows=rows)
    assert torch.isfinite(out).all()
    assert (out - ref).abs().max().item() <= _tol(ref, K)


@pytest.mark.parametrize("M,N,K,delu", [(1024, 512, 256, True), (1536, 256, 128, False), (300, 256, 128, True),
                                         (1000, 18, 1024, False), (513, 512, 256, True),
                                         (96, 128, 18, True), (3000, 18, 1024, False), (300, 32, 128, False),
                                         (3000, 128, 18, True), (1024, 256, 7, False)])
def test_backward_data_nn(M, N, K, delu):
    g = torch.Generator(device=dev).manual_seed(M + 3 * N + K)
    dY = torch.randn(M, K, device=dev, generator=g)
    W = torch.randn(K, N, device=dev, generator=g) / np.sqrt(K)  # W[out][in] with out = reduction
    H = torch.nn.functional.elu(torch.randn(M, N, device=dev, generator=g))
    ref = dY @ W
    if delu:
        ref = ref * torch.where(H > 0, torch.ones_like(H), H + 1)
    out = torch.empty(M, N, device=dev)
    _gemm(2, 3 if delu else 0, M, N, K, dY, K, W, N, out, N, aux=H if delu else None, ld_aux=N)
    assert (out - ref).abs().max().item() <= _tol(ref, K)


@pytest.mark.parametrize("M,N,K,gather,ldx", [(256, 512, 24576, False, 0), (128, 256, 6000, False, 0),
                                              (18, 128, 4097, False, 0), (256, 630, 24576, True, 0),
                                              (256, 630, 24576, True, 640), (1024, 60, 3000, False, 0),
                                              (12, 128, 96, False, 0), (384, 128, 1024, True, 0),
                                              (1024, 60, 3072, False, 64), (256, 40, 2048, True, 64)])
def test_weight_grad_tn(M, N, K, gather, ldx):
    """dW[o][i] = sum_b dY[b][o] X[b][i] (split over b, partials reduced), db[o] = sum_b dY[b][o].  128-row
    m tiles with 128- (or, for n <= 64, 64-) wide n tiles inside X's row pitch take the LDS-DMA kernel
    (ldx = 640: the padded history pitch; 64: the padded actor/critic input), the others the register-staged one."""
    g = torch.Generator(device=dev).manual_seed(M * N + K)
    dY = torch.randn(K, M, device=dev, generator=g)
    src = K + 11
    ldx = ldx or N
    X = torch.randn(src, ldx, device=dev, generator=g)
    rows = torch.randperm(src, device=dev)[:K].contiguous() if gather else None
    Xk = (X[rows] if gather else X[:K])[:, :N]
    ref = dY.T.double() @ Xk.double()
    out = torch.empty(M, N, device=dev)
    db = torch.empty(M, device=dev)
    ws = torch.empty(64 * (M * N + M) * 2, device=dev)
    _gemm(3, 4, M, N, K, dY, M, X, ldx, out, N, bias=db, rows=rows, ws=ws)
    err = (out.double() - ref).abs().max().item()
    assert err <= 4e-6 * np.sqrt(K) * (ref.abs().max().item() + 1.0), err
    assert (db.double() - dY.double().sum(0)).abs().max().item() <= 1e-5 * np.sqrt(K) * 10


@pytest.mark.parametrize("layout,M,N,K", [(0, 24576, 256, 512), (0, 4096, 1024, 64), (2, 24576, 512, 256),
                                          (3, 256, 512, 24576), (0, 300, 200, 60), (2, 333, 200, 50),
                                          (3, 300, 100, 5000)])
def test_x6_error_is_fp32_class(layout, M, N, K):
    """Products whose tiles fit the split-bf16 kernel (csrc/lrl_gemm.hip gemm_x6_kernel: x = hi + mid + lo exactly,
    six bf16 MFMA products, fp32 accumulation): the error against an fp64 product, relative to sum_k |a b|, stays at
    the fp32 level (<= 1e-6 here; the fp32 MFMA measures 1.6-2.4e-7 on the same shapes, the x6 kernel 1.6-2.1e-7),
    for interior tiles and for ragged m / n / k edges."""
    g = torch.Generator(device=dev).manual_seed(M + N + K + layout)
    if layout == 0:
        A = torch.randn(M, K, device=dev, generator=g)
        W = torch.randn(N, K, device=dev, generator=g) * 0.1
        out = torch.empty(M, N, device=dev)
        _gemm(0, 0, M, N, K, A, K, W, K, out, N)
        ref = A.double() @ W.double().T
        mag = A.double().abs() @ W.double().abs().T
    elif layout == 2:
        A = torch.randn(M, K, device=dev, generator=g)
        W = torch.randn(K, N, device=dev, generator=g) * 0.1
        out = torch.empty(M, N, device=dev)
        _gemm(2, 0, M, N, K, A, K, W, N, out, N)
        ref = A.double() @ W.double()
        mag = A.double().abs() @ W.double().abs()
    else:
        dY = torch.randn(K, M, device=dev, generator=g)
        X = torch.randn(K, N, device=dev, generator=g) * 0.1
        out = torch.empty(M, N, device=dev)
        db = torch.empty(M, device=dev)
        ws = torch.empty(64 * (M * N + M) * 2, device=dev)
        _gemm(3, 4, M, N, K, dY, M, X, N, out, N, bias=db, ws=ws)
        ref = dY.double().T @ X.double()
        mag = dY.double().abs().T @ X.double().abs()
        assert ((db.double() - dY.double().sum(0)).abs() / dY.double().abs().sum(0)).max().item() <= 1e-6
    rel = ((out.double() - ref).abs() / mag).max().item()
    assert rel <= 1e-6, rel


@pytest.mark.parametrize("layout,epi,M,N,K,gather", [(0, 2, 24576, 256, 512, False), (0, 2, 4096, 1024, 64, False),
                                                     (0, 1, 1024, 128, 256, False), (0, 2, 2048, 256, 640, True),
                                                     (0, 0, 192, 384, 48, False), (2, 3, 24576, 512, 256, False),
                                                     (2, 3, 1024, 256, 32, False), (2, 0, 640, 256, 128, False)])
def test_pre_split_weight_kernel_is_bit_identical(layout, epi, M, N, K, gather):
    """The LDS-DMA pre-split-B kernel (gemm_x6p_kernel: weights split into bf16 planes once, layout | 0x100) gives the
    same bits as gemm_x6_kernel (fp32 B split while staging): same split, same six products in the same k order."""
    g = torch.Generator(device=dev).manual_seed(M + N + K + epi)
    src = torch.randn(M + 50 if gather else M, K, device=dev, generator=g)
    rows = torch.randperm(M + 50, device=dev, generator=g)[:M].contiguous() if gather else None
    W = torch.randn(N, K, device=dev, generator=g) if layout == 0 else torch.randn(K, N, device=dev, generator=g)
    ldb = K if layout == 0 else N
    bias = torch.randn(N, device=dev, generator=g)
    aux = torch.randn(M, N, device=dev, generator=g) if epi == 3 else None
    ws = torch.empty(3 * N * ((K + 15) // 16 * 16), device=dev)
    c0, c1 = torch.empty(M, N, device=dev), torch.full((M, N), float("nan"), device=dev)
    _gemm(layout, epi, M, N, K, src, K, W, ldb, c0, N, bias=bias, aux=aux, ld_aux=N, rows=rows)
    _gemm(layout | 0x100, epi, M, N, K, src, K, W, ldb, c1, N, bias=bias, aux=aux, ld_aux=N, rows=rows, ws=ws)
    assert torch.equal(c0, c1), (c0 - c1).abs().max().item()


@pytest.mark.parametrize("M,N,K,ldx,gather", [(256, 512, 24576, 512, False), (128, 256, 24576, 256, False),
                                              (128, 128, 4096, 128, False), (256, 256, 3000 * 16, 256, False),
                                              (256, 630, 24576, 640, True), (128, 200, 8192, 256, False),
                                              (128, 60, 4096, 128, True), (1024, 60, 24576, 64, False),
                                              (256, 40, 8192, 64, True)])
def test_lds_dma_weight_gradient_is_bit_identical(M, N, K, ldx, gather):
    """The LDS-DMA weight-gradient kernel (gemm_x6t_kernel) against gemm_x6_kernel (lrl_debug_gemm_paths(2) turns it
    off): the split-k partials and the bias-gradient partials, hence the reduced dW / db, are bit-identical — also for
    a ragged n inside the row pitch and for gathered rows (the adaptation layer's history)."""
    g = torch.Generator(device=dev).manual_seed(M + N + K)
    dY = torch.randn(K, M, device=dev, generator=g)
    Xs = torch.randn(K + 77 if gather else K, ldx, device=dev, generator=g)
    rows = torch.randperm(K + 77, device=dev, generator=g)[:K].contiguous() if gather else None
    X = (Xs[rows] if gather else Xs)[:, :N]
    ws = torch.empty(256 * (M * N + M), device=dev)
    outs = []
    lib = _abi.lib()
    for mask in (2, 0):
        prev = lib.lrl_debug_gemm_paths(C.c_int32(mask))
        try:
            out, db = torch.empty(M, N, device=dev), torch.empty(M, device=dev)
            _gemm(3, 4, M, N, K, dY, M, Xs, ldx, out, N, bias=db, rows=rows, ws=ws)
            outs.append((out, db))
        finally:
            lib.lrl_debug_gemm_paths(C.c_int32(prev))
    assert torch.equal(outs[0][0], outs[1][0]), (outs[0][0] - outs[1][0]).abs().max().item()
    assert torch.equal(outs[0][1], outs[1][1])
    ref = dY.double().T @ X.double()
    mag = dY.double().abs().T @ X.double().abs()
    assert ((outs[1][0].double() - ref).abs() / mag).max().item() <= 1e-6


@pytest.mark.parametrize("layout,epi,M,N,K,gather", [(0, 2, 24576, 256, 512, False), (0, 2, 4096, 1024, 64, False),
                                                     (0, 1, 24576, 128, 256, False), (0, 2, 4096, 256, 640, True),
                                                     (0, 0, 192, 384, 48, False), (2, 3, 24576, 512, 256, False),
                                                     (2, 3, 4096, 256, 32, False), (2, 0, 640, 256, 128, False),
                                                     (2, 3, 8192, 64, 128, False), (0, 2, 8192, 64, 96, True)])
def test_lds_dma_batch_products_are_bit_identical(layout, epi, M, N, K, gather):
    """The LDS-DMA forward / backward-data kernel (gemm_x6d_kernel) against gemm_x6_kernel (lrl_debug_gemm_paths(4)
    turns it off) on the same tile shapes: bit-identical outputs for every epilogue, gathered rows, 64 / 128 tiles."""
    g = torch.Generator(device=dev).manual_seed(M + N + K + epi + layout)
    src = torch.randn(M + 50 if gather else M, K, device=dev, generator=g)
    rows = torch.randperm(M + 50, device=dev, generator=g)[:M].contiguous() if gather else None
    W = torch.randn(N, K, device=dev, generator=g) if layout == 0 else torch.randn(K, N, device=dev, generator=g)
    ldb = K if layout == 0 else N
    bias = torch.randn(N, device=dev, generator=g)
    aux = torch.randn(M, N, device=dev, generator=g) if epi == 3 else None
    lib = _abi.lib()
    outs = []
    for mask in (4, 8):  # (bit 3: the forward products on the x6d kernel too, as LRL_GEMM_X6D=2)
        prev = lib.lrl_debug_gemm_paths(C.c_int32(mask))
        try:
            c = torch.full((M, N), float("nan"), device=dev)
            _gemm(layout, epi, M, N, K, src, K, W, ldb, c, N, bias=bias, aux=aux, ld_aux=N, rows=rows)
            outs.append(c)
        finally:
            lib.lrl_debug_gemm_paths(C.c_int32(prev))
    assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max().item()
