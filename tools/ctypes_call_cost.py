"""Cost of one ctypes call into libsgp from Python with torch imported (as in bench.py): a
CFUNCTYPE (releases the GIL around the call) against a PYFUNCTYPE (keeps it), on
sgp_vi_red1_count (pure host arithmetic).  usage: python3 tools/ctypes_call_cost.py"""
import ctypes as C
import os
import sys
import timeit

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401  (bench.py's process has it, with its threads)
    from sparsergps_amd import _lib
    L = _lib.lib()
    addr = C.cast(L.sgp_vi_red1_count, C.c_void_p).value
    cf = C.CFUNCTYPE(C.c_int64, C.c_int64)(addr)
    pf = C.PYFUNCTYPE(C.c_int64, C.c_int64)(addr)
    n = 200000
    for name, f in (("CFUNCTYPE", cf), ("PYFUNCTYPE", pf), ("CFUNCTYPE", cf)):
        t = timeit.timeit(lambda: f(256), number=n) / n
        print(f"{name}: {1e6 * t:.2f} us per call")
    import numpy as np
    U = np.random.rand(256, 3)
    th = np.random.rand(5)
    for label, fn in (("np.asfortranarray(U) copy", lambda: np.asfortranarray(U)),
                      ("np.zeros(6)", lambda: np.zeros(6)),
                      ("arr.ctypes.data", lambda: th.ctypes.data),
                      ("np.exp(np.sin(np.arange(5)))", lambda: np.exp(np.sin(np.arange(5))))):
        t = timeit.timeit(fn, number=n) / n
        print(f"{label}: {1e6 * t:.2f} us")
    import torch as T
    if T.cuda.is_available():
        T.zeros(1, device="cuda")   # torch's GPU threads started
        for name, f in (("CFUNCTYPE (cuda init)", cf), ("PYFUNCTYPE (cuda init)", pf)):
            t = timeit.timeit(lambda: f(256), number=n) / n
            print(f"{name}: {1e6 * t:.2f} us per call")


if __name__ == "__main__":
    main()
