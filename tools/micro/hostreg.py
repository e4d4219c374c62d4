"""A/B for the FASTQ reader's host side: DMA straight from the file's pages
(mmap + hipHostRegister, whole file or per chunk) against the pread-into-pinned-buffers copy.
Writes a 3.2-GB synthetic file into /dev/shm, times each way of getting its bytes into HBM.
usage: python tools/micro/hostreg.py [GB]"""
import ctypes
import mmap
import os
import sys
import threading
import time

import numpy as np
import torch

GB = float(sys.argv[1]) if len(sys.argv) > 1 else 3.2
hip = ctypes.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
H2D = 1
REG_MAPPED, REG_RO = 0x2, 0x8


def ok(rc, what):
    if rc != 0:
        raise RuntimeError("%s failed: %d" % (what, rc))


path = "/dev/shm/skq_hostreg.bin"
n = int(GB * 1e9) & ~(4095)
with open(path, "wb") as f:
    blk = os.urandom(1 << 20) * 64
    left = n
    while left:
        m = min(left, len(blk))
        f.write(blk[:m])
        left -= m
torch.cuda.init()
dev = torch.empty(n, dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
fd = os.open(path, os.O_RDONLY)
try:
    for rep in range(2):
        # 1. whole file: mmap (populated), register, one copy
        t0 = time.perf_counter()
        mm = mmap.mmap(fd, n, mmap.MAP_SHARED | getattr(mmap, "MAP_POPULATE", 0), mmap.PROT_READ)
        t1 = time.perf_counter()
        # (a read-only mapping cannot back ctypes' from_buffer; numpy gives its address)
        mv = memoryview(mm)
        arr = np.frombuffer(mv, dtype=np.uint8)
        addr = arr.ctypes.data
        rc = hip.hipHostRegister(ctypes.c_void_p(addr), n, REG_MAPPED | REG_RO)
        t2 = time.perf_counter()
        ok(rc, "hipHostRegister")
        ok(hip.hipMemcpyAsync(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(addr), n, H2D, ctypes.c_void_p(st)), "copy")
        ok(hip.hipStreamSynchronize(ctypes.c_void_p(st)), "sync")
        t3 = time.perf_counter()
        ok(hip.hipHostUnregister(ctypes.c_void_p(addr)), "unregister")
        t4 = time.perf_counter()
        print("whole-file register: mmap %.3f s, register %.3f s (%.1f GB/s), copy %.3f s (%.1f GB/s), unregister %.3f s;"
              " total %.3f s = %.1f GB/s" % (t1 - t0, t2 - t1, n / (t2 - t1) / 1e9, t3 - t2, n / (t3 - t2) / 1e9,
                                             t4 - t3, t4 - t0, n / (t4 - t0) / 1e9), flush=True)
        del arr, mv
        mm.close()

        # 2. per-chunk register + copy, T threads over the file
        for T, CH in ((4, 64 << 20), (8, 64 << 20), (8, 256 << 20)):
            mm = mmap.mmap(fd, n, mmap.MAP_SHARED, mmap.PROT_READ)
            mv = memoryview(mm)
            arr = np.frombuffer(mv, dtype=np.uint8)
            base = arr.ctypes.data
            chunks = [(o, min(CH, n - o)) for o in range(0, n, CH)]
            err = []

            def work(i):
                s = torch.cuda.Stream()
                try:
                    for j in range(i, len(chunks), T):
                        o, m = chunks[j]
                        ok(hip.hipHostRegister(ctypes.c_void_p(base + o), m, REG_MAPPED | REG_RO), "register")
                        ok(hip.hipMemcpyAsync(ctypes.c_void_p(dev.data_ptr() + o), ctypes.c_void_p(base + o), m, H2D,
                                              ctypes.c_void_p(s.cuda_stream)), "copy")
                        ok(hip.hipStreamSynchronize(ctypes.c_void_p(s.cuda_stream)), "sync")
                        ok(hip.hipHostUnregister(ctypes.c_void_p(base + o)), "unregister")
                except Exception as e:  # noqa: BLE001
                    err.append(e)

            t0 = time.perf_counter()
            th = [threading.Thread(target=work, args=(i,)) for i in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            t1 = time.perf_counter()
            if err:
                raise err[0]
            print("chunked register+copy: %d threads x %d MiB: %.3f s = %.1f GB/s" % (T, CH >> 20, t1 - t0, n / (t1 - t0) / 1e9),
                  flush=True)
            del arr, mv
            mm.close()

        # 3. pread into pinned buffers + copy (the reader's current way), T threads
        for T, CH in ((12, 32 << 20),):
            pins = [torch.empty(CH, dtype=torch.uint8).pin_memory() for _ in range(T)]
            chunks = [(o, min(CH, n - o)) for o in range(0, n, CH)]

            def work2(i):
                s = torch.cuda.Stream()
                pb = pins[i]
                pa = pb.data_ptr()
                view = (ctypes.c_char * CH).from_address(pa)
                for j in range(i, len(chunks), T):
                    o, m = chunks[j]
                    got = os.preadv(fd, [memoryview(view)[:m]], o)
                    assert got == m
                    ok(hip.hipMemcpyAsync(ctypes.c_void_p(dev.data_ptr() + o), ctypes.c_void_p(pa), m, H2D,
                                          ctypes.c_void_p(s.cuda_stream)), "copy")
                    ok(hip.hipStreamSynchronize(ctypes.c_void_p(s.cuda_stream)), "sync")

            t0 = time.perf_counter()
            th = [threading.Thread(target=work2, args=(i,)) for i in range(T)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            t1 = time.perf_counter()
            print("pread+pinned copy: %d threads x %d MiB: %.3f s = %.1f GB/s" % (T, CH >> 20, t1 - t0, n / (t1 - t0) / 1e9),
                  flush=True)
finally:
    os.close(fd)
    os.unlink(path)
