"""Per-call latency and host CPU of cc_page_crc_host's lanes (engine.hip
page_crc_lane), each configuration in a fresh child process, native caller
threads (bench.run_scan_ops).  Round 6 ran it over the lane's completion-wait
variants ($CC_LANE_WAIT 0 host function + condvar, 1 blocking-sync event, 2/4
stream-written word polled with the default / a 1 us timer slack, 3
hipStreamSynchronize; $CC_LANE_HOSTOUT: CRCs stored straight to pinned memory),
profiles/lane_wait_ab_r06*.jsonl; the engine kept 4 + hostout (the knobs are
gone: the env pairs now only label the lines).  Per variant:
one thread's latency and CPU (calling thread, whole process) per call at 4 KiB /
4 MiB / 16 MiB, and 10 threads' ScanChunkRequest mix (metapage + 4 x 4 MiB).
usage: python scripts/lane_wait_ab.py [out.jsonl]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch
    import bench
    T = 10
    fb = 4096 + (16 << 20)
    hs = [torch.empty(fb, dtype=torch.uint8, pin_memory=True).random_(0, 256) for _ in range(T)]
    bufs = [h.numpy() for h in hs]
    res = {"wait": os.environ.get("CC_LANE_WAIT", "0"), "hostout": os.environ.get("CC_LANE_HOSTOUT", "0")}
    for size in (4096, 4 << 20, 16 << 20):
        n = 64 if size > 4096 else 400
        bench.run_scan_ops(bufs[:1], [4096], [size], 8, "gpu")
        _, _, want, _, _ = bench.run_scan_ops(bufs[:1], [4096], [size], 1, "cpu")
        rc, lat, crcs, wall, cpu = bench.run_scan_ops(bufs[:1], [4096], [size], n, "gpu")
        res[str(size)] = {"rc": rc, "us_p50": round(float(np.median(lat)), 1),
                          "thread_cpu_us": round(cpu / n * 1e6, 1),
                          "process_cpu_us": round(bench.run_scan_ops.last_process_cpu_s / n * 1e6, 1),
                          "ok": bool((crcs == want[0, 0]).all())}
    offs = [0] + [4096 + k * (4 << 20) for k in range(4)]
    lens = [4096] + [4 << 20] * 4
    calls = 300
    bench.run_scan_ops(bufs, offs, lens, 10, "gpu")
    _, _, want, _, _ = bench.run_scan_ops(bufs, offs, lens, 5, "cpu")
    rc, lat, crcs, wall, cpu = bench.run_scan_ops(bufs, offs, lens, calls, "gpu")
    tot = sum(lens) / 5 * calls * T
    res["10threads"] = {"rc": rc, "agg_GiBps": round(tot / 2**30 / wall, 2),
                        "process_cpu_s_per_GiB": round(bench.run_scan_ops.last_process_cpu_s / (tot / 2**30), 4),
                        "thread_cpu_s_per_GiB": round(cpu / (tot / 2**30), 4),
                        "ok": bool(all((crcs[t] == np.resize(want[t], calls)).all() for t in range(T)))}
    print(json.dumps(res), flush=True)


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    lines = []
    pairs = [tuple(x.split(",")) for x in os.environ.get("LANE_AB", "4,1").split()]
    for wait, hostout in pairs:
        env = dict(os.environ, CC_LANE_WAIT=wait, CC_LANE_HOSTOUT=hostout)
        r = subprocess.run([sys.executable, __file__, "child"], env=env, capture_output=True, text=True, timeout=240)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        lines.append(line[-1] if line else json.dumps({"wait": wait, "hostout": hostout, "rc": r.returncode,
                                                       "err": r.stderr[-800:]}))
        print(lines[-1], flush=True)
    if out:
        with open(out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    child() if sys.argv[1:2] == ["child"] else main()
