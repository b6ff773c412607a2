"""Does a blocking wait burn the calling thread's CPU?  (diagnostic)
Prints caller thread CPU time vs wall time for: torch.cuda.synchronize() behind
~50 ms of kernels, and cc_page_crc_host over 2 GiB of pinned memory."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from curve_amd import crc as C  # noqa: E402


def timed(fn):
    w, c = time.perf_counter(), time.thread_time()
    fn()
    return round(time.perf_counter() - w, 4), round(time.thread_time() - c, 4)


def main():
    if os.environ.get("SPIN_PROBE_FLAGS"):
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        rc = hip.hipSetDeviceFlags(int(os.environ["SPIN_PROBE_FLAGS"]))
        print(json.dumps({"hipSetDeviceFlags": int(os.environ["SPIN_PROBE_FLAGS"]), "rc": rc}))
    d = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
    d.random_(0, 256)
    out = torch.empty(d.numel() // 4096, dtype=torch.int32, device="cuda")
    C.page_crc(d, 4096, out=out)
    torch.cuda.synchronize()

    def kernels_then_sync():
        for _ in range(80):
            C.page_crc(d, 4096, out=out)
        torch.cuda.synchronize()

    print(json.dumps({"what": "torch.cuda.synchronize behind kernels", "wall_cpu": timed(kernels_then_sync)}))
    h = torch.empty(2 << 30, dtype=torch.uint8, pin_memory=True)
    h[:] = 7
    a = h.numpy()
    C.page_crc_host(a[: 1 << 20], 4096)
    print(json.dumps({"what": "cc_page_crc_host pinned 2 GiB", "wall_cpu": timed(lambda: C.page_crc_host(a, 4096))}))
    print(json.dumps({"what": "cc_page_crc_host pageable 512 MiB",
                      "wall_cpu": timed(lambda: C.page_crc_host(a[: 512 << 20].copy(), 4096))}))


if __name__ == "__main__":
    main()
