"""Diagnostic (round 6): does a one-rank RCCL communicator's grouped self ncclSend/ncclRecv
deliver every byte of one large message?  Round 5's C1 exchange (knn_comm.cpp) sent a rank's own
1.2 GB record block to itself as ONE grouped send/recv and got only its first half.  This script
takes the library out of the picture: it drives RCCL directly (ctypes, the same librccl.so.1 the
library dlopens) on torch buffers with a known pattern (src[i] = i), for message sizes around
2^29 .. 2^31 bytes and the datatypes int32 / int8, and prints one JSON line per case: how many
elements arrived intact and where the first wrong one is.  Optionally (--chunks) each message is
sent as pieces of at most CHUNK elements inside the same group, the exchange's round-6 plan.

    python scripts/diag_rccl_self.py [--sizes-mb 256,1024,1200,2100] [--chunk-mi 64]
"""
import argparse
import ctypes
import json
import sys
import time

import torch

NCCL_INT8, NCCL_INT32 = 0, 2


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


def load_rccl():
    for name in ("librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"):
        try:
            lib = ctypes.CDLL(name, mode=ctypes.RTLD_GLOBAL)
            break
        except OSError:
            continue
    else:
        raise SystemExit("RCCL not found")
    P = ctypes.c_void_p
    lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(UniqueId)]
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(P), ctypes.c_int, UniqueId, ctypes.c_int]
    lib.ncclSend.argtypes = [P, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, P, P]
    lib.ncclRecv.argtypes = [P, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, P, P]
    lib.ncclCommDestroy.argtypes = [P]
    lib.ncclGetVersion.argtypes = [ctypes.POINTER(ctypes.c_int)]
    return lib


def rccl_path():
    with open("/proc/self/maps") as f:
        for line in f:
            if "librccl" in line:
                return line.split()[-1]
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes-mb", default="256,600,1024,1100,1200,1600,2100")
    ap.add_argument("--chunk-mi", type=int, default=0, help="also run each size as pieces of this many Mi elements")
    args = ap.parse_args()
    lib = load_rccl()
    ver = ctypes.c_int()
    lib.ncclGetVersion(ctypes.byref(ver))
    torch.cuda.set_device(0)
    uid = UniqueId()
    assert lib.ncclGetUniqueId(ctypes.byref(uid)) == 0
    comm = ctypes.c_void_p()
    assert lib.ncclCommInitRank(ctypes.byref(comm), 1, uid, 0) == 0
    stream = torch.cuda.current_stream().cuda_stream
    print(json.dumps({"rccl_version": ver.value, "rccl_file": rccl_path(), "torch": torch.__version__}), flush=True)
    plans = [0] + ([args.chunk_mi << 20] if args.chunk_mi else [])
    for mb in (int(x) for x in args.sizes_mb.split(",")):
        nbytes = mb * 1_000_000
        for dt, esz in ((NCCL_INT32, 4), (NCCL_INT8, 1)):
            n = nbytes // esz
            if dt == NCCL_INT32:
                src = torch.arange(n, dtype=torch.int32, device="cuda")
                dst = torch.full((n,), -1, dtype=torch.int32, device="cuda")
            else:
                src = (torch.arange(n, dtype=torch.int64, device="cuda") % 251).to(torch.int8)
                dst = torch.full((n,), -1, dtype=torch.int8, device="cuda")
            for chunk in plans:
                dst.fill_(-1)
                torch.cuda.synchronize()
                step = chunk if chunk else n
                t0 = time.perf_counter()
                assert lib.ncclGroupStart() == 0
                msgs = 0
                for o in range(0, n, step):
                    c = min(step, n - o)
                    assert lib.ncclSend(src.data_ptr() + o * esz, c, dt, 0, comm, stream) == 0
                    assert lib.ncclRecv(dst.data_ptr() + o * esz, c, dt, 0, comm, stream) == 0
                    msgs += 1
                rc = lib.ncclGroupEnd()
                torch.cuda.synchronize()
                ms = 1e3 * (time.perf_counter() - t0)
                eq = dst == src
                good = int(eq.sum().item())
                bad = (~eq).nonzero()
                first_bad = int(bad[0].item()) if bad.numel() else None
                print(json.dumps({"bytes": n * esz, "dtype": "int32" if dt == NCCL_INT32 else "int8", "count": n,
                                  "messages": msgs, "group_end": rc, "intact": good, "all_intact": good == n,
                                  "first_bad_elem": first_bad,
                                  "first_bad_byte": None if first_bad is None else first_bad * esz,
                                  "ms": round(ms, 2)}), flush=True)
            del src, dst
            torch.cuda.empty_cache()
    lib.ncclCommDestroy(comm)


if __name__ == "__main__":
    sys.exit(main())
