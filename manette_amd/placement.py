"""Host-thread placement of one rank (SURVEY §8(e) multi-GPU; the reference's runners.py:11-18
starts `ew` emulator processes per learner and leaves their placement to the OS).

One process per GPU runs `ew` native emulator threads (manette_amd/csrc/runner.cpp) plus its own
host thread, which spins on the sampled actions every macro-step. Eight ranks on one node start
8 x (ew + 1) busy threads; left to the scheduler they migrate across NUMA nodes and, when the
node's cores (or the container's CPU quota) are fewer than that, time-slice against each other
on the macro-step's critical path. plan() decides, per rank:
  * the cpu pool: the allowed cpus (sched_getaffinity) on the NUMA node of the rank's GPU (its PCI
    device's numa_node), split in contiguous slices between the local ranks whose GPUs share that
    node — so a rank's threads sit next to its GPU's PCIe root and never on another rank's cores;
  * the thread budget: min(slice, container quota / local ranks); when ew + 1 threads do not fit
    it, ew is capped to budget - 1 (at least 1; the env -> worker split changes, every env's
    trajectory does not) and idle workers spin 50 us instead of 2 ms before sleeping, so an idle
    pool yields its cores to the other ranks' pools;
  * the placement itself, by mode:
      'slice': the rank's host thread and every thread it starts afterwards (the emulator workers)
               may run anywhere in the rank's slice — NUMA-local, disjoint from the other ranks, and
               the scheduler still moves a thread off a core another process keeps busy;
      'pin':   the host thread on the slice's first cpu (plus any cpus no worker takes), worker w on
               the next ones, one cpu each (mh_runner_set_threads);
      'auto':  'slice' when several ranks share the node, else 'off' (the scheduler's placement);
      'off':   nothing changed ('on' is an alias of 'pin').
    One cpu per thread measured badly on the shared 1-GPU boxes (profiles/r06pin: Breakout FiGAR
    273-278k pinned vs 342-523k unpinned, its workers' staging 122-126 vs 32-67 us per step: a pinned
    worker cannot leave a core another tenant keeps busy), so the default keeps the scheduler free
    inside the rank's slice.
plan() is a pure function of the topology it is given (tests/test_placement_cpu.py); topology()
reads it from /proc, /sys and torch on the running host.
"""
import math
import os

SPIN_US = 2000          # runner.cpp kSpinUs: idle spin before the futex sleep
SPIN_US_OVERSUB = 50    # when the rank's threads exceed its share of the node's cores


def parse_cpulist(text):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11] (the kernel's cpulist format)."""
    out = []
    for part in text.strip().split(','):
        if not part:
            continue
        if '-' in part:
            a, b = part.split('-')
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def format_cpulist(cpus):
    """[0, 1, 2, 3, 8] -> '0-3,8'."""
    cpus = sorted(set(cpus))
    parts, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        parts.append(str(cpus[i]) if i == j else '%d-%d' % (cpus[i], cpus[j]))
        i = j + 1
    return ','.join(parts)


def cgroup_cpu_limit(path='/sys/fs/cgroup/cpu.max'):
    """CPUs' worth of the container's CFS quota (cgroup v2 'quota period'), or None if unlimited."""
    try:
        quota, period = open(path).read().split()[:2]
    except (OSError, ValueError):
        return None
    if quota == 'max':
        return None
    return int(quota) / float(period)


def _read(path):
    try:
        return open(path).read().strip()
    except OSError:
        return None


def gpu_numa_node(device_index):
    """NUMA node of GPU device_index's PCI function (None when the host does not report one)."""
    import torch
    p = torch.cuda.get_device_properties(device_index)
    bdf = '%04x:%02x:%02x.0' % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
    v = _read('/sys/bus/pci/devices/%s/numa_node' % bdf)
    if v is None or int(v) < 0:
        return None
    return int(v)


def numa_cpus(node):
    v = _read('/sys/devices/system/node/node%d/cpulist' % node)
    return parse_cpulist(v) if v else []


def topology(local_world):
    """The running host's inputs of plan(): allowed cpus, the quota, each local rank's GPU node
    (device index = local rank, as bench.py / train.py set it; None when this process sees fewer
    devices than local ranks) and the cpus of those nodes."""
    import torch
    allowed = sorted(os.sched_getaffinity(0))
    nodes = [None] * local_world
    try:
        if torch.cuda.device_count() >= local_world:
            nodes = [gpu_numa_node(d) for d in range(local_world)]
    except Exception:  # (no GPU / no PCI information: placement falls back to the allowed set)
        nodes = [None] * local_world
    node_cpus = {n: numa_cpus(n) for n in set(nodes) if n is not None}
    return dict(allowed=allowed, quota=cgroup_cpu_limit(), node_of_rank=nodes, node_cpus=node_cpus)


def plan(ew, E, local_rank, local_world, allowed, quota=None, node_of_rank=None, node_cpus=None, mode='auto'):
    """Placement of local rank `local_rank` of `local_world` (see the module docstring). Returns a
    dict: pinned, ew_used, worker_cpus, main_cpus, spin_us and the report fields."""
    ew_req = max(1, min(int(ew), int(E)))
    node_of_rank = list(node_of_rank) if node_of_rank is not None else [None] * local_world
    node_cpus = node_cpus or {}
    me = node_of_rank[local_rank] if local_rank < len(node_of_rank) else None
    allowed = sorted(allowed)
    if me is not None and set(node_cpus.get(me, [])) & set(allowed):
        pool = [c for c in allowed if c in set(node_cpus[me])]
        group = [r for r in range(local_world) if node_of_rank[r] == me]
    else:  # unknown topology: the allowed cpus, split between every local rank
        pool, group = allowed, list(range(local_world))
    k, idx = len(group), group.index(local_rank)
    lo, hi = (len(pool) * idx) // k, (len(pool) * (idx + 1)) // k
    mine = pool[lo:hi] or pool[idx % len(pool):idx % len(pool) + 1]
    budget = len(mine)
    if quota:  # the container's CPU quota, shared by every local rank
        budget = min(budget, max(1, int(math.floor(quota / max(local_world, 1)))))
    if mode == 'on':
        mode = 'pin'
    eff = ('slice' if local_world > 1 else 'off') if mode == 'auto' else mode
    pinned, sliced = eff == 'pin', eff == 'slice'
    placed = pinned or sliced
    oversub = budget < ew_req + 1
    ew_used = max(1, min(ew_req, budget - 1)) if (placed and oversub) else ew_req
    spin = SPIN_US_OVERSUB if oversub and placed else SPIN_US
    if len(mine) >= ew_used + 1:
        main_cpus = [mine[0]] + mine[1 + ew_used:]
        worker_cpus = mine[1:1 + ew_used]
    else:  # fewer cpus than threads: workers round-robin over the slice, the host thread on all of it
        main_cpus = list(mine)
        worker_cpus = [mine[(1 + w) % len(mine)] for w in range(ew_used)]
    return dict(mode=mode, placement=eff, pinned=pinned, sliced=sliced, numa_node=me, local_rank=local_rank,
                local_world=local_world, cpus=format_cpulist(mine), cores_per_rank=budget, quota=quota,
                ew_requested=int(ew), ew_used=ew_used, threads_per_rank=ew_used + 1, oversubscribed=oversub,
                spin_us=spin, worker_cpus=worker_cpus if pinned else [],
                main_cpus=main_cpus if pinned else (list(mine) if sliced else []))


def apply_before_workers(p):
    """'slice': restrict the calling (host) thread to the rank's slice before the emulator workers
    start, so they inherit it (threads started later do too)."""
    if p['sliced'] and p['main_cpus']:
        os.sched_setaffinity(0, set(p['main_cpus']))


def apply_main(p):
    """'pin': the calling (host) thread onto its cpus, after the workers were pinned to theirs."""
    if p['pinned'] and p['main_cpus']:
        os.sched_setaffinity(0, set(p['main_cpus']))


def report(p):
    """The plan's fields for the bench line (no cpu lists of the workers)."""
    keys = ('mode', 'placement', 'numa_node', 'local_world', 'cpus', 'cores_per_rank', 'quota', 'ew_requested',
            'ew_used', 'threads_per_rank', 'oversubscribed', 'spin_us')
    return {k: p[k] for k in keys}
