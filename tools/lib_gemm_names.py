"""torch.mm (ROCm BLAS library, fp32) on the config-2 step's layer products, for
`rocprofv3 --kernel-trace --stats -- python3 tools/lib_gemm_names.py`: the library's kernel names
(macro tile, matrix instruction, depth) beside the rates of tools/gemm_bench.py --lib.
"""
import torch

SHAPES = [(62464, 1024, 1024), (62464, 512, 1024), (32768, 512, 512), (32768, 1024, 128), (32768, 256, 512)]


def main():
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda:0")
    for M, N, K in SHAPES:
        X = torch.randn(M, K, device=dev)
        W = torch.randn(N, K, device=dev)
        dY = torch.randn(M, N, device=dev)
        for _ in range(3):
            torch.mm(X, W.t())          # forward
            torch.mm(dY, W)             # dgrad
            torch.mm(dY.t(), X)         # wgrad
        torch.cuda.synchronize()
        print(M, N, K, "done", flush=True)


if __name__ == "__main__":
    main()
