"""Known-byte kernels for the FETCH_SIZE / WRITE_SIZE calibration (tools/pmc_calib.hip).

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_cal_f -o cal -- python3 tools/pmc_calib.py
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_cal_w -o cal -- python3 tools/pmc_calib.py
    python3 tools/rocpd_summary.py calib <fetch.db> <write.db> profiles/<tag>_pmc_calib.json

Each kernel moves exactly 512 MiB (twice the 256 MiB Infinity Cache) three times.
"""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NFLOATS = 1 << 27                                   # 512 MiB


def main():
    import torch
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "libpmc_calib.so"))
    lib.pmc_calib_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
    buf = torch.randn(NFLOATS, device="cuda")
    sink = torch.zeros(1 << 20, device="cuda")
    for which in range(5):
        for _ in range(3):
            assert lib.pmc_calib_run(which, ctypes.c_void_p(buf.data_ptr()), NFLOATS,
                                     ctypes.c_void_p(sink.data_ptr())) == 0
        torch.cuda.synchronize()
    print("calibration kernels done", flush=True)


if __name__ == "__main__":
    main()
