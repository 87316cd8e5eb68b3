#!/usr/bin/env python3
"""Root-cause probe for the launch-time ramp of back-to-back C3 launches.

Round 1 saw 1 GiB blocks-kernel launches drift 0.17 -> 0.24 -> 0.17 ms over
the first ~60 launches of a process (VERDICT r01 "weak" 3).  This probe times
every launch with HIP events on the launch stream and, in a sampler thread,
reads the GPU's DPM levels (sclk / mclk / fclk / socclk: the '*' line of
pp_dpm_*) and hwmon power/temperature from sysfs every ~2 ms, so each launch
can be matched with the clock state it ran under.  Phases:

  A  fresh arena, first launches of the process   (clock ramp + first touch)
  B  after 1 s idle, same arena                    (idle -> busy: clocks only)
  C  a second, freshly allocated arena             (first touch, clocks warm)
  D  after 3 s idle, same arena                    (longer idle)
  E  after a 2 s back-to-back settle               (steady state)

Writes gpurun_out/ramp/ramp.json and prints a one-line summary per phase.
"""
import glob
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "leveldb-rs_amd"))


def card_dir(torch):
    """sysfs device dir of cuda:0 (matched by PCI bus id when torch exposes it)."""
    cards = sorted(glob.glob("/sys/class/drm/card*/device"))
    cards = [c for c in cards if os.path.exists(os.path.join(c, "pp_dpm_sclk"))]
    try:
        p = torch.cuda.get_device_properties(0)
        bus = getattr(p, "pci_bus_id", None)
        dom = getattr(p, "pci_domain_id", 0)
        dev = getattr(p, "pci_device_id", 0)
        if bus is not None:
            tag = f"{dom:04x}:{bus:02x}:{dev:02x}."
            for c in cards:
                if os.path.basename(os.path.realpath(c)).startswith(tag):
                    return c, "pci-match"
    except Exception:  # noqa: BLE001 - diagnostics only
        pass
    return (cards[0], "first-card") if cards else (None, "none")


def read_star(path):
    try:
        with open(path) as f:
            for line in f:
                if "*" in line:
                    return line.split(":", 1)[1].replace("*", "").strip()
    except OSError:
        return None
    return None


def read_int(path):
    try:
        with open(path) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return None


class Sampler(threading.Thread):
    def __init__(self, cdir):
        super().__init__(daemon=True)
        self.cdir = cdir
        self.samples = []
        self.stop = False
        hw = glob.glob(os.path.join(cdir, "hwmon", "hwmon*")) if cdir else []
        self.hw = hw[0] if hw else None

    def run(self):
        while not self.stop:
            s = {"t": time.perf_counter()}
            if self.cdir:
                for k in ("sclk", "mclk", "fclk", "socclk"):
                    s[k] = read_star(os.path.join(self.cdir, f"pp_dpm_{k}"))
            if self.hw:
                s["power_uW"] = read_int(os.path.join(self.hw, "power1_average")) or read_int(
                    os.path.join(self.hw, "power1_input"))
                s["temp_mC"] = read_int(os.path.join(self.hw, "temp1_input"))
            self.samples.append(s)
            time.sleep(0.002)


def main():
    import torch
    import lvgpu
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lvgpu.device_init()
    cdir, how = card_dir(torch)
    samp = Sampler(cdir)
    samp.start()
    n, bl = 262144, 4096
    stream = torch.cuda.current_stream()

    def new_arena():
        a = torch.empty(n * bl, dtype=torch.uint8, device=dev)
        lvgpu.fill_splitmix(a, 0, 0x4C444231)
        return a

    out = torch.empty(n, dtype=torch.int32, device=dev)
    phases = {}

    def run(name, arena, launches):
        torch.cuda.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(launches)]
        h0 = time.perf_counter()
        ev0.record(stream)
        for a, b in evs:
            a.record(stream)
            lvgpu.batch_strided(arena, bl, bl, n, out=out, stream=stream)
            b.record(stream)
        torch.cuda.synchronize()
        ms = [a.elapsed_time(b) for a, b in evs]
        ends = [ev0.elapsed_time(b) for _, b in evs]
        phases[name] = {"host_t0": h0, "launch_ms": [round(x, 4) for x in ms],
                        "end_ms": [round(x, 3) for x in ends]}
        k = len(ms)
        q = lambda lo, hi: sum(ms[lo:hi]) / max(1, len(ms[lo:hi]))  # noqa: E731
        print(f"{name}: first10 {q(0, 10):.4f} 10-60 {q(10, 60):.4f} 60-120 {q(60, 120):.4f} "
              f"last100 {q(k - 100, k):.4f} max {max(ms):.4f} at {ms.index(max(ms))}", flush=True)

    arena = new_arena()
    run("A_fresh_process", arena, 600)
    time.sleep(1.0)
    run("B_after_1s_idle", arena, 300)
    arena2 = new_arena()
    run("C_fresh_arena", arena2, 300)
    del arena2
    time.sleep(3.0)
    run("D_after_3s_idle", arena, 300)
    t_end = time.perf_counter() + 2.0
    settle = 0
    while time.perf_counter() < t_end:
        for _ in range(50):
            lvgpu.batch_strided(arena, bl, bl, n, out=out, stream=stream)
        torch.cuda.synchronize()
        settle += 50
    run("E_after_2s_settle", arena, 300)
    samp.stop = True
    samp.join()
    os.makedirs(os.path.join(ROOT, "gpurun_out", "ramp"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "ramp", "ramp.json"), "w") as f:
        json.dump({"card": cdir, "card_match": how, "settle_launches_E": settle, "phases": phases,
                   "samples": samp.samples}, f)
    print(f"card {cdir} ({how}); {len(samp.samples)} sysfs samples", flush=True)


if __name__ == "__main__":
    main()
