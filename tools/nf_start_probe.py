"""Start tools/build/dev_probe back to back, as the GPU suite starts its NFs.

The NF binary (tests/test_gpu_app.py) twice exited at start in round 5 with HIP's
"no ROCm-capable device is detected", on boxes where the runs before and after
saw the GPU.  This probe repeats the start many times in the suite's shape -- the
parent process holds a GPU context (torch), the probe is started from a
forkserver child that never touched the GPU -- and records every start: whether
HIP saw the device, how long the probe's KFD entry outlived its exit, and, on a
failure, the library's description of what the process saw.  The box runs in a
PID namespace and /sys/class/kfd/kfd/proc lists host pids, so a probe's entry is
the one that appears while it holds its context (--hold seconds).  Two modes, alternating:
  wait    the next start waits until the previous probe's KFD entry is gone;
  nowait  the next start follows the previous exit at once.

  python tools/nf_start_probe.py --starts 120 --out gpurun_out/nf_start_probe.jsonl
"""
import argparse
import json
import multiprocessing
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tools", "build", "dev_probe")
KFD = "/sys/class/kfd/kfd/proc"


def kfd_pids():
    try:
        return sorted(int(x) for x in os.listdir(KFD) if x.isdigit())
    except OSError:
        return None


def run_starts(n, out, hold):
    recs = []
    for i in range(n):
        mode = "wait" if i % 2 == 0 else "nowait"
        before = kfd_pids()
        t0 = time.time()
        # the probe holds its context for --hold seconds, so its KFD entry (a
        # host pid: the box runs in a PID namespace) can be told from the others
        p = subprocess.Popen([PROBE, str(hold)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        mine = None
        while p.poll() is None and mine is None and hold > 0:
            new = sorted(set(kfd_pids() or []) - set(before or []))
            if len(new) == 1:
                mine = new[0]
            time.sleep(0.01)
        stdout, stderr = p.communicate(timeout=60)
        t_exit = time.time()
        try:
            r = json.loads(stdout.strip().splitlines()[-1])
        except (ValueError, IndexError):
            r = {"ok": False, "stage": "output", "stdout": stdout[-500:]}
        r.update({"i": i, "mode": mode, "returncode": p.returncode, "wall_s": round(t_exit - t0, 3),
                  "kfd_before": before, "stderr": stderr[-500:]})
        r["kfd_pid"] = mine
        gone_s = None
        if mine is not None:
            r["kfd_listed_at_exit"] = mine in (kfd_pids() or [])
        if mode == "wait" and mine is not None:
            while time.time() - t_exit < 15:
                if mine not in (kfd_pids() or []):
                    gone_s = round(time.time() - t_exit, 3)
                    break
                time.sleep(0.005)
        r["kfd_gone_after_s"] = gone_s
        recs.append(r)
        with open(out, "a") as f:
            f.write(json.dumps(r) + "\n")
        print(json.dumps({k: r.get(k) for k in ("i", "mode", "ok", "init_s", "wall_s", "kfd_gone_after_s")}),
              flush=True)
    return recs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--starts", type=int, default=120)
    ap.add_argument("--hold", type=float, default=0.3, help="seconds each probe keeps its context before exiting")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "nf_start_probe.jsonl"))
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    ctx = multiprocessing.get_context("forkserver")
    ctx.set_forkserver_preload([])
    # the parent holds a GPU context from here on, as the pytest process does
    import torch
    x = torch.zeros(1 << 20, device="cuda")
    torch.cuda.synchronize()
    print(json.dumps({"parent_pid": os.getpid(), "parent_pid_listed": os.getpid() in (kfd_pids() or []),
                      "kfd_pids": kfd_pids()}), flush=True)
    with ctx.Pool(1) as pool:
        recs = pool.apply(run_starts, (args.starts, args.out, args.hold))
    del x
    fails = [r for r in recs if not r.get("ok")]
    waits = [r["kfd_gone_after_s"] for r in recs if r.get("kfd_gone_after_s") is not None]
    summary = {"starts": len(recs), "failures": len(fails),
               "failure_modes": sorted({r["mode"] for r in fails}),
               "kfd_gone_after_s_max": max(waits) if waits else None,
               "kfd_gone_after_s_median": sorted(waits)[len(waits) // 2] if waits else None,
               "kfd_pid_identified": sum(r.get("kfd_pid") is not None for r in recs),
               "kfd_listed_at_exit": sum(bool(r.get("kfd_listed_at_exit")) for r in recs),
               "init_s_max": max((r.get("init_s") or 0) for r in recs)}
    print(json.dumps(summary), flush=True)
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
