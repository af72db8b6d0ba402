"""Run the calibration kernels (tools/calib/pmc_calib.hip, built into libcalib.so by
`make -C tools/calib`) on a 512 MiB buffer -- larger than the 256 MiB Infinity Cache, so
every launch streams from HBM -- 3 launches each; rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE around this script gives the counter per known byte count."""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "libcalib.so"))
    lib.calib_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                              ctypes.c_void_p]
    n = (512 << 20) // 4
    dev = torch.device("cuda", 0)
    buf = torch.ones(n, device=dev)
    scratch = torch.zeros(4096, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    which = [int(a) for a in sys.argv[1:]] or [0, 1, 2]
    for w in which:
        for _ in range(3):
            assert lib.calib_run(w, buf.data_ptr(), n, scratch.data_ptr(), st) == 0
    torch.cuda.synchronize()
    print("calibration launches done: bytes per launch", n * 4)


if __name__ == "__main__":
    main()
