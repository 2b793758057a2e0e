"""Feasibility: does a weight-gradient GEMM on a side stream overlap with the persistent GRU
recurrence (which is latency-bound and leaves most MFMA cycles idle)?"""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "deepspeech.pytorch_amd"))
import torch
from ds2amd import ops, _lib

dev = torch.device("cuda")
T, N, H, D = 501, 32, 800, 2
g = torch.Generator(device="cpu").manual_seed(0)
xproj = torch.randn(T, N, D, 3 * H, device=dev) * 0.1
whf = torch.randn(3 * H, H, device=dev) * 0.03
whr = torch.randn(3 * H, H, device=dev) * 0.03
bhf = torch.zeros(3 * H, device=dev); bhr = torch.zeros(3 * H, device=dev)
lens = torch.full((N,), T, dtype=torch.int32, device=dev)
h_all = torch.empty(T, N, D, H, device=dev)
gates = torch.empty(T, N, D, 4 * H, device=dev)
ws = torch.empty(_lib.size("ds2_gru_fwd_workspace_size", N, H, D), dtype=torch.uint8, device=dev)
# a dW-like GEMM: [2400 x 800] = A^T[16032 x 2400]^T @ B[16032 x 800]
A = torch.randn(T * N, 3 * H, device=dev); B = torch.randn(T * N, H, device=dev)
C = torch.empty(3 * H, H, device=dev)

def rec(stream):
    with torch.cuda.stream(stream):
        _lib.call("ds2_gru_fwd", T, N, H, D, xproj.data_ptr(), whf.data_ptr(), whr.data_ptr(),
                  bhf.data_ptr(), bhr.data_ptr(), lens.data_ptr(), h_all.data_ptr(),
                  gates.data_ptr(), ws.data_ptr(), ws.numel(), stream.cuda_stream)

def gemm(stream, reps):
    with torch.cuda.stream(stream):
        for _ in range(reps):
            ops.sgemm(A, B, C, m=3 * H, n=H, k=T * N, trans_a=True, lda=3 * H, ldb=H, ldc=H)

s1 = torch.cuda.Stream(); s2 = torch.cuda.Stream()
def timed(fn):
    torch.cuda.synchronize(); t0 = time.perf_counter(); fn(); torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3
for _ in range(2):
    timed(lambda: rec(s1)); timed(lambda: gemm(s2, 1))
for reps in (2, 4, 8):
    tr = timed(lambda: rec(s1))
    tg = timed(lambda: gemm(s2, reps))
    def both():
        rec(s1)          # recurrence first (its WGs dispatch first)
        gemm(s2, reps)
    tb = timed(both)
    print(f"reps {reps}: recurrence {tr:.2f} ms, gemm x{reps} {tg:.2f} ms, serial {tr+tg:.2f}, "
          f"concurrent {tb:.2f} ms -> hidden {tr+tg-tb:.2f} ms")
