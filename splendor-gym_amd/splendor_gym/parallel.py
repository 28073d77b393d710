"""Multi-GPU sharding: one process per GPU, tables split by contiguous global id ranges.

Tables are independent games, so the step path never communicates.  The only
collective is at report time: an all-gather of per-table episode-return sums and episode counts
(torch.distributed; backend "nccl" is RCCL over xGMI on ROCm, "gloo" for CPU tests).  Every RNG
stream is keyed by the GLOBAL table id, so per-table results are identical for 1/2/4/8 GPUs.
"""
import os

import torch
import torch.distributed as dist


def shard_range(n_global, rank, world):
    """[lo, hi) global table ids owned by `rank` (contiguous, sizes differ by at most one)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, extra = divmod(int(n_global), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def init_distributed(backend=None):
    """Initialise the default process group from torchrun's env (RANK, WORLD_SIZE, LOCAL_RANK,
    MASTER_ADDR/PORT).  Returns (rank, world, local_rank); (0, 1, 0) without a launcher.
    Backend: `backend`, else $SPLENDOR_DIST_BACKEND, else nccl (RCCL) with GPUs, gloo without.
    gloo with GPUs rehearses several ranks on one card (local_device maps ranks onto the cards)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        if backend is None:
            backend = os.environ.get("SPLENDOR_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return rank, world, local


def local_device(local):
    """The GPU of local rank `local`: one per rank on a full node; ranks share cards when there
    are more ranks than cards (gloo rehearsal)."""
    return torch.device("cuda", local % max(1, torch.cuda.device_count()))


def device_identity(device):
    """The physical GPU behind `device` as a string that two processes on one node compare equal
    exactly when they drive the same card: host name + PCI domain:bus:device when torch exposes them,
    else the device UUID, else the visible index (with HIP_VISIBLE_DEVICES, which differs per process)."""
    import socket
    props = torch.cuda.get_device_properties(device)
    pci = [getattr(props, a, None) for a in ("pci_domain_id", "pci_bus_id", "pci_device_id")]
    if all(isinstance(v, int) for v in pci):
        ident = "pci %04x:%02x:%02x" % tuple(pci)
    elif getattr(props, "uuid", None) is not None:
        ident = f"uuid {props.uuid}"
    else:
        ident = f"index {torch.device(device).index} of HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES', '')}"
    return f"{socket.gethostname()}/{ident}"


def device_census(identity):
    """Every rank's device identity (device_identity), gathered on every rank: how many ranks, how
    many DISTINCT devices they run on, and whether any two share one (a rehearsal of N ranks on fewer
    cards is not an N-GPU figure)."""
    if _single():
        ids = [identity]
    else:
        ids = [None] * dist.get_world_size()
        dist.all_gather_object(ids, identity)
    distinct = len(set(ids))
    return {"ranks": len(ids), "devices": distinct, "shared_device": distinct < len(ids), "identities": ids}


def _single():
    """No process group, or a group of one rank: the collectives below return their input."""
    return not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1


def _host_collectives():
    """gloo collectives run on host tensors here (its CUDA support is partial)."""
    return dist.get_backend() == "gloo"


def gather_returns(ep_return, ep_count, n_global=None):
    """All-gather per-table (return sum, episode count) shards into full [n_global] tensors on
    every rank.  Shards may differ in size by one (shard_range); they are padded to equal
    length for all_gather_into_tensor and trimmed after."""
    if _single():
        return ep_return.clone(), ep_count.clone()
    world = dist.get_world_size()
    if _host_collectives():
        ret, cnt = gather_returns_host(ep_return.cpu(), ep_count.cpu(), n_global)
        return ret.to(ep_return.device), cnt.to(ep_count.device)
    n_local = torch.tensor([ep_return.numel()], dtype=torch.int64, device=ep_return.device)
    sizes = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(sizes, n_local)
    sizes = [int(s.item()) for s in sizes]
    width = max(sizes)
    packed = torch.zeros((2, width), dtype=torch.float64, device=ep_return.device)
    packed[0, :ep_return.numel()] = ep_return.to(torch.float64)
    packed[1, :ep_count.numel()] = ep_count.to(torch.float64)
    out = torch.empty((world * 2, width), dtype=torch.float64, device=ep_return.device)
    dist.all_gather_into_tensor(out, packed)  # rank-major concatenation along dim 0
    out = out.view(world, 2, width)
    ret = torch.cat([out[r, 0, :sizes[r]] for r in range(world)])
    cnt = torch.cat([out[r, 1, :sizes[r]] for r in range(world)])
    if n_global is not None and ret.numel() != n_global:
        raise RuntimeError(f"gathered {ret.numel()} tables, expected {n_global}")
    return ret.to(torch.float32), cnt.to(torch.int64)


def gather_returns_host(ep_return, ep_count, n_global=None):
    """gather_returns on host tensors (gloo): same padding and layout."""
    world = dist.get_world_size()
    sizes = [None] * world
    dist.all_gather_object(sizes, int(ep_return.numel()))
    width = max(sizes)
    packed = torch.zeros((2, width), dtype=torch.float64)
    packed[0, :ep_return.numel()] = ep_return.to(torch.float64)
    packed[1, :ep_count.numel()] = ep_count.to(torch.float64)
    parts = [torch.empty_like(packed) for _ in range(world)]
    dist.all_gather(parts, packed)
    ret = torch.cat([parts[r][0, :sizes[r]] for r in range(world)])
    cnt = torch.cat([parts[r][1, :sizes[r]] for r in range(world)])
    if n_global is not None and ret.numel() != n_global:
        raise RuntimeError(f"gathered {ret.numel()} tables, expected {n_global}")
    return ret.to(torch.float32), cnt.to(torch.int64)


def max_over_ranks(value, device=None):
    """Max of a host float over all ranks (the bench's slowest-rank time)."""
    if _single():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=None if _host_collectives() else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None):
    if not _single():
        if device is not None and device.type == "cuda" and not _host_collectives():
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


# env var a self-launched rank carries (launch_local_ranks): the ranks must run on distinct devices
SELF_LAUNCHED_ENV = "SPLENDOR_SELF_LAUNCHED"
# opt-in for a rehearsal of N self-launched ranks on fewer GPUs (the line is then labelled a shared-device
# rehearsal, never a node figure; collectives need SPLENDOR_DIST_BACKEND=gloo, RCCL refuses a shared card)
REHEARSAL_ENV = "SPLENDOR_SHARED_DEVICE_REHEARSAL"


def free_port(addr="127.0.0.1"):
    """A TCP port on `addr` that nothing listens on right now (the rendezvous port of a local group)."""
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def launch_local_ranks(n, cmd, env=None, port=None, poll_s=0.2, stream=None):
    """Run `cmd` (an argv list) as ranks 0..n-1 of one process group on this node: what
    `torch.distributed.run --nnodes 1 --nproc-per-node n --master-addr 127.0.0.1` does, for a caller
    that was started without a launcher (`python bench.py --gpus 8`).

    Each child gets RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT and
    SPLENDOR_SELF_LAUNCHED=1, inherits stdout / stderr, and picks its own device
    (`local_device(LOCAL_RANK)`): this process never touches a GPU, so the children are started from
    a process without a HIP context.  Waits for all of them; when one exits non-zero the others are
    terminated (their exact PIDs) so none is left waiting in a collective, and so are all of them when
    this process is interrupted or sent SIGTERM.  Returns 0 when every rank exited 0, else the first
    non-zero exit status seen (a signal -s maps to 128 + s)."""
    import signal
    import subprocess
    import sys
    import threading
    import time
    if n < 1:
        raise ValueError("n must be >= 1")
    port = port or free_port()
    base = dict(os.environ if env is None else env)
    base.update(WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    base[SELF_LAUNCHED_ENV] = "1"
    # a SIGTERM to this process (a driver's time limit) ends the children too instead of orphaning them
    main = threading.current_thread() is threading.main_thread()

    def _term(signum, frame):
        raise SystemExit(128 + signum)
    prev = signal.signal(signal.SIGTERM, _term) if main else None
    procs = []
    status = 0
    try:
        for r in range(n):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen(list(cmd), env=e))
        live = list(procs)
        while live:
            time.sleep(poll_s)
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    print(f"rank {procs.index(p)} exited with status {rc}; stopping the other ranks",
                          file=stream or sys.stderr, flush=True)
                    for q in live:
                        q.terminate()
    finally:
        for p in procs:  # normally all have exited; after an exception or a signal, stop the rest (exact PIDs)
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        if main:
            signal.signal(signal.SIGTERM, prev)
    return status


def require_distinct_devices(census, world):
    """A self-launched run (launch_local_ranks) is an N-GPU figure only if its N ranks drove N distinct
    devices: returns the error text when they did not, else None (an external launcher's shared-device
    rehearsal is labelled instead, bench.node_fields)."""
    if os.environ.get(SELF_LAUNCHED_ENV) != "1" or census["devices"] >= world or os.environ.get(REHEARSAL_ENV) == "1":
        return None
    return (f"{world} ranks found only {census['devices']} distinct device(s) ({census['identities']}): "
            f"an N-GPU run needs N GPUs; no figure is reported")
