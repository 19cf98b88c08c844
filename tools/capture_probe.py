"""Which part of a hipGraph capture of PyTorch's process-group all-gather crashes on this stack
(round 4's `bench.py --gather-graph` died with SIGSEGV under torchrun, gpurun_out/r04n).

Each case runs in its own child process (one RCCL rank, world size 1, as the bench's one-GPU
rehearsal) with faulthandler on, so a segfault prints the Python frame it happened in; the parent
prints one line per case: exit code and the last lines of the child's stderr.

  python tools/capture_probe.py            # all cases
  python tools/capture_probe.py CASE       # one case (the child entry point)
"""
import faulthandler
import os
import socket
import subprocess
import sys

CASES = {
    # torch.cuda.graph's default capture_error_mode ("global"): every thread's unsafe calls are
    # checked while the capture is open -- including the process group's watchdog thread
    "pg_all_gather_global": dict(mode="global", eager_first=True),
    "pg_all_gather_thread_local": dict(mode="thread_local", eager_first=True),
    "pg_all_gather_relaxed": dict(mode="relaxed", eager_first=True),
    # the first all-gather of a fresh communicator happens inside the capture (lazy init)
    "pg_all_gather_global_cold": dict(mode="global", eager_first=False),
    "pg_all_gather_thread_local_cold": dict(mode="thread_local", eager_first=False),
}


def child(name):
    faulthandler.enable(all_threads=True)
    import torch
    import torch.distributed as dist
    c = CASES[name]
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    x = torch.arange(1 << 20, dtype=torch.float32, device=dev)
    out = torch.empty_like(x)
    if c["eager_first"]:
        dist.all_gather_into_tensor(out, x)
        torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    print(f"[{name}] capture begins", file=sys.stderr, flush=True)
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s, capture_error_mode=c["mode"]):
            y = x * 2
            dist.all_gather_into_tensor(out, y)
    print(f"[{name}] capture ended", file=sys.stderr, flush=True)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    ok = bool(torch.equal(out, x * 2))
    print(f"[{name}] replayed 10x, result {'equal' if ok else 'DIFFERS'}", file=sys.stderr, flush=True)
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 1:
        child(sys.argv[1])
        return
    for name in CASES:
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        try:
            p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), name], env=env, capture_output=True,
                               text=True, timeout=120)
            rc, err = p.returncode, p.stderr
        except subprocess.TimeoutExpired as e:
            rc, err = "timeout", (e.stderr or b"").decode() if isinstance(e.stderr, bytes) else (e.stderr or "")
        tail = " | ".join(l for l in err.strip().splitlines()[-12:] if l.strip())
        print(f"{name}: exit {rc}: {tail}", flush=True)


if __name__ == "__main__":
    main()
