"""Driver of fetch_calib.hip: one process per (mode, size); run it under rocprofv3 --pmc FETCH_SIZE
(or WRITE_SIZE) and compare the per-dispatch counter with the streamed bytes:
  python3 scripts/micro/fetch_calib.py MODE BYTES REPS"""
import ctypes as C
import os
import sys

lib = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libfetch_calib.so"))
lib.fetch_calib.argtypes = [C.c_int, C.c_size_t, C.c_int]
mode, nbytes, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
rc = lib.fetch_calib(mode, nbytes, reps)
print("rc", rc, "mode", mode, "bytes", nbytes, "reps", reps)
sys.exit(0 if rc == 0 else 1)
