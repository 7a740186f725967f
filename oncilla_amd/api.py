"""Python binding of the libocm C ABI (``csrc/include/oncillamem.h``).

Thin ctypes layer over the in-tree ``build/lib/libocm.so``: the native library
does all the work (mailbox RPC to ocmd, IPC import, gfx950 transfer kernels).
Mirrors the reference app API (reference inc/oncillamem.h:69-89) plus the
MI355X extensions (``ocm_alloc_ex``, async one-sided copies, stats).

    from oncilla_amd import api
    with api.Client() as ocm:
        a = ocm.alloc(api.OCM_REMOTE_GPU, local_bytes=1 << 20, remote_bytes=1 << 20)
        a.fill(seed=1); a.put(0, 0, 1 << 20); a.get(0, 0, 1 << 20)
        assert a.check(seed=1) == 0
        a.free()
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

from .utils.paths import lib_path

OCM_LOCAL_HOST = 1
OCM_LOCAL_RMA = 2
OCM_REMOTE_RMA = 3
OCM_LOCAL_RDMA = 4
OCM_REMOTE_RDMA = 5
OCM_LOCAL_GPU = 6
OCM_REMOTE_GPU = 7

OCM_ALLOC_STRIPE = 1 << 0
OCM_ALLOC_HOST_TIER = 1 << 1
OCM_ALLOC_NO_SPILL = 1 << 2
OCM_ALLOC_ZERO = 1 << 3
OCM_ALLOC_LOOPBACK = 1 << 4

OCM_TIER_HOST = 1
OCM_TIER_GPU = 2
OCM_MAX_EXTENTS = 8

REMOTE_KINDS = (OCM_REMOTE_GPU, OCM_REMOTE_RDMA, OCM_REMOTE_RMA)


class OcmParams(ctypes.Structure):
    """struct ocm_params (48 bytes)."""

    _fields_ = [
        ("src_offset", ctypes.c_uint64),
        ("dest_offset", ctypes.c_uint64),
        ("src_offset_2", ctypes.c_uint64),
        ("dest_offset_2", ctypes.c_uint64),
        ("bytes", ctypes.c_uint64),
        ("op_flag", ctypes.c_int),
    ]


class OcmAllocParams(ctypes.Structure):
    """struct ocm_alloc_params (24 bytes)."""

    _fields_ = [
        ("local_alloc_bytes", ctypes.c_uint64),
        ("rem_alloc_bytes", ctypes.c_uint64),
        ("kind", ctypes.c_int),
    ]


class OcmAllocExParams(ctypes.Structure):
    _fields_ = [
        ("remote_rank", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("stripe_width", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
        ("stripe_unit", ctypes.c_uint64),
    ]


class OcmRemoteInfo(ctypes.Structure):
    _fields_ = [
        ("n_extents", ctypes.c_uint32),
        ("tier", ctypes.c_uint32 * OCM_MAX_EXTENTS),
        ("owner_rank", ctypes.c_int32 * OCM_MAX_EXTENTS),
        ("owner_gpu", ctypes.c_int32 * OCM_MAX_EXTENTS),
        ("extent_bytes", ctypes.c_uint64 * OCM_MAX_EXTENTS),
        ("stripe_unit", ctypes.c_uint64),
        ("alloc_id", ctypes.c_uint64),
        ("remote_bytes", ctypes.c_uint64),
        ("net_mask", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]


class OcmDaemonStats(ctypes.Structure):
    _fields_ = [
        ("rank", ctypes.c_int32),
        ("gpu", ctypes.c_int32),
        ("num_nodes", ctypes.c_int32),
        ("num_apps", ctypes.c_int32),
        ("gpu_capacity", ctypes.c_uint64),
        ("gpu_used", ctypes.c_uint64),
        ("host_capacity", ctypes.c_uint64),
        ("host_used", ctypes.c_uint64),
        ("n_alloc", ctypes.c_uint64),
        ("n_free", ctypes.c_uint64),
        ("n_reclaimed", ctypes.c_uint64),
        ("n_spilled", ctypes.c_uint64),
        ("n_slabs", ctypes.c_uint64),
        ("ctrl_ticks", ctypes.c_uint64),
        ("n_leases", ctypes.c_uint64),
        ("lease_allocs", ctypes.c_uint64),
        ("xgmi_peers", ctypes.c_uint32),
        ("min_hops", ctypes.c_uint16),
        ("max_hops", ctypes.c_uint16),
        ("ctrl_transport", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]

    def as_dict(self) -> dict:
        d = {name: getattr(self, name) for name, _ in self._fields_ if name != "reserved"}
        d["ctrl"] = CTRL_TRANSPORTS.get(d["ctrl_transport"], "unknown")
        return d


# ocm_daemon_stats.ctrl_transport
CTRL_TRANSPORTS = {0: "tcp", 1: "socket", 2: "rccl", 3: "tcp (left ticks)", 4: "starting"}


class OcmError(RuntimeError):
    pass


_lib = None
_lib_lock = threading.Lock()


def load(path: Optional[str] = None) -> ctypes.CDLL:
    """Load libocm.so once (fails loudly if it has not been built)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        p = path or lib_path()
        if not os.path.exists(p):
            raise OcmError(f"{p} not found: build the native tree first (python -c 'import __graft_entry__ as g; g.build()')")
        lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        sigs = {
            "ocm_init": (i32, []),
            "ocm_tini": (i32, []),
            "ocm_alloc": (vp, [ctypes.POINTER(OcmAllocParams)]),
            "ocm_alloc_ex": (vp, [ctypes.POINTER(OcmAllocParams), ctypes.POINTER(OcmAllocExParams)]),
            "ocm_free": (i32, [vp]),
            "ocm_localbuf": (i32, [vp, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_size_t)]),
            "ocm_is_remote": (ctypes.c_bool, [vp]),
            "ocm_alloc_kind": (i32, [vp]),
            "ocm_remote_sz": (i32, [vp, ctypes.POINTER(ctypes.c_size_t)]),
            "ocm_copy_out": (i32, [vp, vp]),
            "ocm_copy_in": (i32, [vp, vp]),
            "ocm_copy": (i32, [vp, vp, ctypes.POINTER(OcmParams)]),
            "ocm_copy_onesided": (i32, [vp, ctypes.POINTER(OcmParams)]),
            "ocm_copy_onesided_async": (i32, [vp, ctypes.POINTER(OcmParams)]),
            "ocm_wait": (i32, [vp]),
            "ocm_copy_onesided_batch": (i32, [vp, ctypes.POINTER(OcmParams), i32, i32]),
            "ocm_stream_wait": (i32, [vp, vp]),
            "ocm_plan_create": (vp, []),
            "ocm_plan_add": (i32, [vp, vp, ctypes.POINTER(OcmParams), i32]),
            "ocm_plan_launch": (i32, [vp, vp]),
            "ocm_plan_destroy": (i32, [vp]),
            "ocm_stream_signal": (i32, [vp, vp]),
            "ocm_remote_info": (i32, [vp, ctypes.POINTER(OcmRemoteInfo)]),
            "ocm_remotebuf": (vp, [vp]),
            "ocm_stats": (i32, [i32, ctypes.POINTER(OcmDaemonStats)]),
            "ocm_rank": (i32, []),
            "ocm_num_nodes": (i32, []),
            "ocm_device": (i32, []),
            "ocm_last_error": (ctypes.c_char_p, []),
            "ocm_x_layout": (None, [ctypes.POINTER(u64)]),
            "ocm_x_xfer": (i32, [i32, vp, ctypes.POINTER(vp), i32, u64, u64, u64, i32, i32, i32, i32]),
            "ocm_x_time_device_copy": (ctypes.c_double, [i32, vp, vp, u64, i32, i32, i32, i32]),
            "ocm_x_time_onesided": (ctypes.c_double, [vp, ctypes.POINTER(OcmParams), i32]),
            "ocm_x_time_onesided_samples": (i32, [vp, ctypes.POINTER(OcmParams), i32, i32, u64, u64,
                                                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64)]),
            "ocm_x_alloc_latency": (i32, [ctypes.POINTER(OcmAllocParams), ctypes.POINTER(OcmAllocExParams), i32,
                                          ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
            "ocm_x_pattern": (ctypes.c_longlong, [vp, u64, u64, ctypes.c_uint32, i32]),
            "ocm_x_counters": (None, [ctypes.POINTER(u64)]),
            "ocm_x_service_stats": (None, [ctypes.POINTER(u64)]),
            "ocm_x_service_health": (None, [ctypes.POINTER(u64)]),
            "ocm_x_tick_stats": (ctypes.c_int, [ctypes.POINTER(u64)]),
            "ocm_x_quiesce": (None, []),
            "ocm_x_service_trace": (i32, [ctypes.POINTER(u64), i32]),
            "ocm_x_service_pages": (i32, [ctypes.c_void_p, ctypes.POINTER(u64)]),
            "ocm_x_adam": (i32, [vp, vp, vp, u64, u64, u64, ctypes.POINTER(ctypes.c_float), vp]),
            "ocm_x_adam_multi": (i32, [vp, i32, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(u64),
                                       ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64),
                                       ctypes.POINTER(ctypes.c_float), i32, vp]),
            "ocm_x_adam_bf16": (i32, [vp, vp, vp, u64, u64, u64, u64, ctypes.POINTER(ctypes.c_float), vp]),
            "ocm_x_set_tuning": (None, [i32, i32, i32]),
            "ocm_x_set_tuning_dir": (i32, [i32, i32, i32, i32]),
            "ocm_x_batch": (i32, [i32, vp, ctypes.POINTER(vp), i32, u64, ctypes.POINTER(u64), i32, i32]),
            "ocm_x_link_info": (i32, [i32, i32, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]),
            "ocm_x_extent_handle": (i32, [vp, i32, ctypes.c_char_p]),
            "ocm_x_extent_region": (i32, [vp, i32, ctypes.POINTER(u64)]),
            "ocm_x_xgmi_diag": (None, [ctypes.POINTER(u64)]),
            "ocm_x_link_layout": (None, [ctypes.POINTER(u64)]),
            "ocm_x_ipc_open": (i32, [i32, ctypes.c_char_p, ctypes.POINTER(vp)]),
            "ocm_x_ipc_close": (i32, [i32, vp]),
            "ocm_x_pattern_dev": (ctypes.c_longlong, [i32, vp, u64, u64, ctypes.c_uint32, i32]),
            "ocm_x_torch_pool_config": (None, [i32, ctypes.c_uint32]),
            "ocm_x_torch_pool_stats": (None, [ctypes.POINTER(u64)]),
        }
        for name, (res, args) in sigs.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def _adam_hp(hp) -> tuple:
    """(b1, b2, eps, weight_decay, step_size, 1/sqrt(bias_correction2)[, decay]) -> 7 floats.
    decay is AdamW's weight multiplier 1 - lr * weight_decay; NaN (the default) selects
    L2-regularised Adam."""
    hp = tuple(float(x) for x in hp)
    if len(hp) not in (6, 7):
        raise ValueError("Adam hyper-parameters: 6 values (Adam) or 7 (AdamW decay multiplier last)")
    return hp if len(hp) == 7 else hp + (float("nan"),)


def last_error() -> str:
    e = load().ocm_last_error()
    return e.decode(errors="replace") if e else ""


COUNTER_KEYS = ["n_put", "n_get", "bytes_put", "bytes_get", "n_alloc", "n_free", "n_copy", "bytes_copy", "ns_put",
                "ns_get", "ns_alloc", "ns_free", "n_batch", "n_batch_ops", "bytes_batch", "ns_batch",
                "n_batch_launches", "n_slab_fd", "n_slab_path", "n_link_rpc", "n_link_wake"]
OCM_BATCH_ASYNC = 1


class Plan:
    """A fixed transfer schedule replayed as one HIP graph launch (ocm_plan_*).

    plan.add(alloc, ops) appends a stage (ops as for Allocation.batch); stages run in order.
    plan.launch() blocks; plan.launch(stream) queues on a torch stream / hipStream_t handle.
    """

    def __init__(self, client: "Client"):
        self._c = client
        self.handle = client.lib.ocm_plan_create()
        if not self.handle:
            raise OcmError("ocm_plan_create: " + last_error())
        self._keep = []

    def add(self, alloc: "Allocation", ops) -> "Plan":
        arr = ops if isinstance(ops, BatchOps) else batch_ops(ops)
        if self._c.lib.ocm_plan_add(self.handle, alloc.handle, arr.array, arr.n) != 0:
            raise OcmError("ocm_plan_add: " + last_error())
        return self

    def launch(self, stream=None) -> None:
        h = None
        if stream is not None:
            h = ctypes.c_void_p(stream if isinstance(stream, int) else stream.cuda_stream)
        if self._c.lib.ocm_plan_launch(self.handle, h) != 0:
            raise OcmError("ocm_plan_launch: " + last_error())

    def close(self) -> None:
        if self.handle:
            self._c.lib.ocm_plan_destroy(self.handle)
            self.handle = None

    def __enter__(self) -> "Plan":
        return self

    def __exit__(self, *exc) -> None:
        self.close()


class BatchOps:
    """A prepared descriptor list for Allocation.batch (ctypes array of ocm_params)."""

    def __init__(self, array, n: int):
        self.array = array
        self.n = n


def batch_ops(ops) -> BatchOps:
    """Descriptor list from (op_flag, local_offset, remote_offset, nbytes) tuples, or from an
    (n, 4) integer array with those columns (vectorised, no per-op Python objects)."""
    try:
        import numpy as np
    except ImportError:  # pragma: no cover
        np = None
    if np is not None and isinstance(ops, np.ndarray):
        n = int(ops.shape[0])
        mat = np.zeros((max(1, n), 6), dtype=np.uint64)  # struct ocm_params: 6 x u64
        if n:
            mat[:n, 0] = ops[:, 1]  # src_offset  (local)
            mat[:n, 1] = ops[:, 2]  # dest_offset (remote)
            mat[:n, 4] = ops[:, 3]  # bytes
            mat[:n, 5] = ops[:, 0]  # op_flag
        b = BatchOps(mat.ctypes.data_as(ctypes.POINTER(OcmParams)), n)
        b.keep = mat
        return b
    ops = list(ops)
    arr = (OcmParams * max(1, len(ops)))()
    for i, (flag, loff, roff, n) in enumerate(ops):
        arr[i] = OcmParams(loff, roff, 0, 0, n, flag)
    return BatchOps(arr, len(ops))


def set_tuning(variant: int = 0, blocks: int = 0, nontemporal: bool = True) -> None:
    """Transfer-kernel tuning for this process (0 auto / 1 register / 2 LDS-DMA; grid cap; nt stores)."""
    load().ocm_x_set_tuning(variant, blocks, 1 if nontemporal else 0)


def set_tuning_dir(op_flag: int, variant: int = 0, blocks: int = 0, nontemporal=True) -> None:
    """Per-direction override for one-sided kernel ops (op_flag 0 get, 1 put); variant 0 clears it.
    ``nontemporal``: True / 1 nt stores, False / 0 plain, 2 write-through (sc1) loads and stores
    in the register kernel. ``set_tuning`` clears both overrides."""
    nt = 2 if nontemporal == 2 else (1 if nontemporal else 0)
    if load().ocm_x_set_tuning_dir(op_flag, variant, blocks, nt) != 0:
        raise ValueError(f"bad tuning: op_flag={op_flag} variant={variant} blocks={blocks}")


def link_info(dev: int, peer: int) -> Optional[dict]:
    """xGMI/PCIe link type and hop count between two visible devices (hipExtGetLinkTypeAndHopCount)."""
    t, h = ctypes.c_uint32(), ctypes.c_uint32()
    if load().ocm_x_link_info(dev, peer, ctypes.byref(t), ctypes.byref(h)) != 0:
        return None
    return {"type": int(t.value), "hops": int(h.value)}


def counters() -> dict:
    """This process's libocm operation counters."""
    out = (ctypes.c_uint64 * len(COUNTER_KEYS))()
    load().ocm_x_counters(out)
    return dict(zip(COUNTER_KEYS, [int(v) for v in out]))


def link_layout() -> dict:
    """Byte layout of the app <-> daemon shared-memory link (ocm/shmlink.h), for tests."""
    out = (ctypes.c_uint64 * 11)()
    load().ocm_x_link_layout(out)
    keys = ("bytes", "req_taken", "rsp_taken", "daemon_polling", "app_waiting", "req", "rsp", "slot", "seq", "slots",
            "magic")
    return dict(zip(keys, (int(x) for x in out)))


def xgmi_diag() -> dict:
    """This process's xGMI self-diagnosis: its device, the peers it enabled access to,
    and the other GPUs' HBM slabs it imported (or was refused) over IPC, and how many
    push-get kernels it launched on owners' GPUs."""
    out = (ctypes.c_uint64 * 5)()
    load().ocm_x_xgmi_diag(out)
    return {"device": ctypes.c_int64(out[0]).value, "peer_access": int(out[1]), "ipc_imports": int(out[2]),
            "ipc_failures": int(out[3]), "push_launches": int(out[4])}


def quiesce() -> None:
    """Park this process's resident copy service now. Optional: on the library's
    AQL queues (the default) a device-wide synchronize never waits for the
    service; on HIP streams (OCM_SERVICE_QUEUE=hip) the service leaves by itself
    OCM_SERVICE_IDLE_US (50 us) after its last op, so torch.cuda.synchronize right
    after a small blocking op waits at most that long, and quiesce() removes even
    that wait. The next op relaunches the service. No-op without a GPU or before
    any op."""
    load().ocm_x_quiesce()


def service_stats() -> dict:
    """Copy-service diagnostics of this process: ops served, mean host time to post a
    request, mean host wait for its completion, mean GPU time from doorbell seen to
    completion published (microseconds), and how many times it was relaunched after
    leaving on its idle timeout (OCM_SERVICE_IDLE_US)."""
    out = (ctypes.c_uint64 * 5)()
    load().ocm_x_service_stats(out)
    n = int(out[0])
    return {"ops": n, "post_us": out[1] / n / 1e3 if n else None, "wait_us": out[2] / n / 1e3 if n else None,
            "gpu_us": out[3] / 100.0 / n if n else None, "relaunches": int(out[4])}


def service_health() -> dict:
    """Copy-service health of this process (ocm/xfer.h roster): gang ops sized below
    the width they wanted because fewer of the service's workgroups were running
    (`degraded`), instances that left with the posted op unfinished and had it
    re-posted (`incomplete_exits`, expected 0), ops abandoned after
    OCM_SERVICE_TIMEOUT_MS and redone by a launch once the instance had drained
    (`aborts`), whether an instance could not be drained at all (`wedged`), the
    smallest roster a gang op was sized to (`roster_min`, 0: none yet), the
    running instance's roster (`roster`, 0: not running), and the relaunches after
    an idle exit with their mean host time (reap + launch, microseconds). `queue`:
    "aql" when the service runs on the library's own AQL queues (a device-wide
    synchronize never waits for it, and its lead may stay resident alone between
    bursts, OCM_SERVICE_LONE_US), "hip" on HIP streams; `promotions`: gang ops that
    replaced a lone lead with a full instance; `lone`: the running instance's lead
    is alone; `drain_max_ms` / `drain_max_site`: the longest wait for a lane's
    workgroups to leave and where it happened."""
    out = (ctypes.c_uint64 * 19)()
    load().ocm_x_service_health(out)
    n, k = int(out[6]), int(out[10])
    return {"degraded": int(out[0]), "incomplete_exits": int(out[1]), "aborts": int(out[2]),
            "wedged": bool(out[3]), "roster_min": int(out[4]), "roster": int(out[5]), "relaunches": n,
            "relaunch_host_us_mean": round(out[7] / n / 1e3, 2) if n else None,
            # every start, split: choosing a lane (runtime stream queries) / the launch call itself
            "start_pick_us_mean": round(out[8] / k / 1e3, 2) if k else None,
            "start_launch_us_mean": round(out[9] / k / 1e3, 2) if k else None,
            "queue": "aql" if out[11] else "hip", "promotions": int(out[12]), "lone": bool(out[13]),
            # the longest wait for a lane's workgroups to leave, and where
            "drain_max_ms": round(out[14] / 1e6, 3),
            "drain_max_site": {0: None, 1: "start", 2: "park", 3: "stop", 4: "abort", 5: "repost"}.get(int(out[15])),
            "overlaps": int(out[16]), "resident": bool(out[17]),
            "lead_xcd": (int(out[18]) & 0xFF) - 1 if out[18] else None,
            # the lead's HW_REG_HW_ID: CU bits 8..11, shader array 12, engine 13..15 (gfx9 layout)
            "lead_hw_id": int(out[18]) >> 8 if out[18] else None}


def tick_stats() -> dict | None:
    """The local daemon's tick control transport (RCCL or socket collective):
    ticks completed, this rank's own records from post to delivery (mean / max
    microseconds) and that hop split into its stages, the mean gap between
    completed ticks, the host time per Collective::start, idle ticks run and TCP
    wake-ups sent. None when the call fails; zeros on a TCP-only daemon."""
    out = (ctypes.c_uint64 * 16)()
    if load().ocm_x_tick_stats(out) != 0:
        return None
    n, p, k, d = int(out[1]), int(out[4]), int(out[6]), int(out[13])
    return {"ticks": int(out[0]), "own_records": n,
            "hop_mean_us": round(out[2] / n / 1e3, 2) if n else None, "hop_max_us": round(out[3] / 1e3, 1),
            # the hop, split: post -> its tick queued (0 when one was already queued),
            # queued -> completion seen by the tick thread, completion -> the event loop took it
            "hop_wait_mean_us": round(out[10] / n / 1e3, 2) if n else None,
            "hop_exec_mean_us": round(out[11] / n / 1e3, 2) if n else None,
            "deliver_mean_us": round(out[12] / d / 1e3, 2) if d else None,
            "tick_period_mean_us": round(out[5] / p / 1e3, 2) if p else None,
            "start_mean_us": round(out[7] / k / 1e3, 2) if k else None, "start_max_us": round(out[8] / 1e3, 1),
            "transport": int(out[9] & 0xFFFFFFFF), "ticks_per_start": int(out[9] >> 32),
            "idle_ticks": int(out[14]), "tcp_wakes": int(out[15])}


def service_totals() -> dict:
    """Raw cumulative copy-service counters (diff two snapshots for a breakdown)."""
    out = (ctypes.c_uint64 * 5)()
    load().ocm_x_service_stats(out)
    return {"ops": int(out[0]), "ns_post": int(out[1]), "ns_wait": int(out[2]), "gpu_ticks": int(out[3]),
            "relaunches": int(out[4])}


def service_breakdown(before: dict, after: dict) -> Optional[dict]:
    """Per-op means between two service_totals() snapshots: host time to post the
    request, GPU time from doorbell seen to completion published, and the rest of
    the host's wait (the two PCIe crossings: doorbell read, completion write)."""
    n = after["ops"] - before["ops"]
    if n <= 0:
        return None
    post = (after["ns_post"] - before["ns_post"]) / n / 1e3
    wait = (after["ns_wait"] - before["ns_wait"]) / n / 1e3
    gpu = (after["gpu_ticks"] - before["gpu_ticks"]) / n / 100.0
    return {"ops": n, "post_us": round(post, 3), "gpu_us": round(gpu, 3), "crossings_us": round(wait - gpu, 3),
            "relaunches": after["relaunches"] - before["relaunches"]}


def service_trace(n_wgs: int = 32) -> list:
    """Copy-service phase stamps of the last request, per workgroup (needs the TRACE bit,
    16, in OCM_SERVICE_PROTO): microseconds of [seen, copy start, drained, counted/done]
    relative to workgroup 0's doorbell-seen stamp; None for a workgroup that never stamped."""
    out = (ctypes.c_uint64 * (4 * n_wgs))()
    if load().ocm_x_service_trace(out, n_wgs) != 0:
        raise OcmError("ocm_x_service_trace: no copy service running")
    t0 = out[0]
    rows = []
    for w in range(n_wgs):
        r = out[4 * w:4 * w + 4]
        rows.append(None if r[0] == 0 else [round((x - t0) / 100.0, 2) if x else None for x in r])
    return rows


def layout() -> dict:
    out = (ctypes.c_uint64 * 8)()
    load().ocm_x_layout(out)
    keys = ["msg", "ocm_params", "ocm_alloc_params", "msg_union_offset", "region", "node_config", "alloc_req",
            "ipc_handle"]
    return dict(zip(keys, [int(v) for v in out]))


class Allocation:
    """An ocm_alloc_t handle."""

    def __init__(self, client: "Client", handle: int, kind: int):
        self._c = client
        self.handle = ctypes.c_void_p(handle)
        self.kind = kind

    # --- reference accessors ---
    def localbuf(self) -> tuple[int, int]:
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        if self._c.lib.ocm_localbuf(self.handle, ctypes.byref(p), ctypes.byref(n)) != 0:
            raise OcmError("ocm_localbuf: " + last_error())
        return (p.value or 0), n.value

    @property
    def local_ptr(self) -> int:
        return self.localbuf()[0]

    @property
    def local_bytes(self) -> int:
        return self.localbuf()[1]

    def is_remote(self) -> bool:
        return bool(self._c.lib.ocm_is_remote(self.handle))

    def remote_size(self) -> int:
        n = ctypes.c_size_t()
        if self._c.lib.ocm_remote_sz(self.handle, ctypes.byref(n)) != 0:
            raise OcmError("ocm_remote_sz: no remote buffer")
        return n.value

    def alloc_kind(self) -> int:
        return int(self._c.lib.ocm_alloc_kind(self.handle))

    def remote_info(self) -> dict:
        info = OcmRemoteInfo()
        if self._c.lib.ocm_remote_info(self.handle, ctypes.byref(info)) != 0:
            raise OcmError("ocm_remote_info: not a remote allocation")
        n = info.n_extents
        return {
            "alloc_id": info.alloc_id,
            "remote_bytes": info.remote_bytes,
            "stripe_unit": info.stripe_unit,
            "extents": [
                {"owner_rank": info.owner_rank[i], "owner_gpu": info.owner_gpu[i], "tier": info.tier[i],
                 "bytes": info.extent_bytes[i], "net": bool(info.net_mask >> i & 1)}
                for i in range(n)
            ],
        }

    def extent_handle(self, i: int = 0) -> bytes:
        """Raw 64-byte export handle of extent i (IPC handle, host-tier path or net: capability)."""
        buf = ctypes.create_string_buffer(64)
        if self._c.lib.ocm_x_extent_handle(self.handle, i, buf) != 0:
            raise OcmError("ocm_x_extent_handle: no such extent")
        return buf.raw

    def extent_region(self, i: int = 0) -> dict:
        """Where extent i sits in its owner's slab (with extent_handle(i), a process on the
        owner's GPU can map the same bytes: see owner_view())."""
        out = (ctypes.c_uint64 * 4)()
        if self._c.lib.ocm_x_extent_region(self.handle, i, out) != 0:
            raise OcmError("ocm_x_extent_region: no such extent")
        return {"offset": int(out[0]), "bytes": int(out[1]), "slab_bytes": int(out[2]),
                "owner_gpu": ctypes.c_int64(out[3]).value}

    # --- data movement ---
    def onesided(self, op_flag: int, local_offset: int, remote_offset: int, nbytes: int, async_: bool = False) -> None:
        p = OcmParams(local_offset, remote_offset, 0, 0, nbytes, op_flag)
        fn = self._c.lib.ocm_copy_onesided_async if async_ else self._c.lib.ocm_copy_onesided
        if fn(self.handle, ctypes.byref(p)) != 0:
            raise OcmError("ocm_copy_onesided: " + last_error())

    def put(self, local_offset: int, remote_offset: int, nbytes: int, async_: bool = False) -> None:
        """One-sided write: local[local_offset:] -> remote[remote_offset:]."""
        self.onesided(1, local_offset, remote_offset, nbytes, async_)

    def get(self, local_offset: int, remote_offset: int, nbytes: int, async_: bool = False) -> None:
        """One-sided read: remote[remote_offset:] -> local[local_offset:]."""
        self.onesided(0, local_offset, remote_offset, nbytes, async_)

    def wait(self) -> None:
        if self._c.lib.ocm_wait(self.handle) != 0:
            raise OcmError("ocm_wait: " + last_error())

    @staticmethod
    def _stream_handle(stream):
        if stream is None:
            import torch

            stream = torch.cuda.current_stream()
        return ctypes.c_void_p(stream if isinstance(stream, int) else stream.cuda_stream)

    def stream_wait(self, stream=None) -> None:
        """Order this allocation's next op after the work queued on `stream` (default: torch's current stream)."""
        if self._c.device < 0:
            return
        if self._c.lib.ocm_stream_wait(self.handle, self._stream_handle(stream)) != 0:
            raise OcmError("ocm_stream_wait: " + last_error())

    def stream_signal(self, stream=None) -> None:
        """Make later work on `stream` (default: torch's current stream) wait for this allocation's async ops."""
        if self._c.device < 0:
            return
        if self._c.lib.ocm_stream_signal(self.handle, self._stream_handle(stream)) != 0:
            raise OcmError("ocm_stream_signal: " + last_error())

    def batch(self, ops, async_: bool = False) -> None:
        """Many one-sided ops in one launch (ocm_copy_onesided_batch).

        ops: iterable of (op_flag, local_offset, remote_offset, nbytes) with op_flag 1 = put,
        0 = get; or a prepared :func:`batch_ops` array (no per-call conversion).
        """
        arr = ops if isinstance(ops, BatchOps) else batch_ops(ops)
        if self._c.lib.ocm_copy_onesided_batch(self.handle, arr.array, arr.n, OCM_BATCH_ASYNC if async_ else 0) != 0:
            raise OcmError("ocm_copy_onesided_batch: " + last_error())

    def adam(self, p, g, m_off: int, v_off: int, hp, stream=None, w_off: Optional[int] = None) -> None:
        """Fused Adam on GPU tensors p/g (contiguous) with exp_avg / exp_avg_sq at byte offsets
        m_off / v_off of the remote half, read and written in place (ocm_x_adam). float32 p/g are
        updated directly; bfloat16 p/g need w_off, the fp32 master weights in the remote half,
        which the update runs on (ocm_x_adam_bf16). hp = (b1, b2, eps, weight_decay, step_size,
        1/sqrt(bias_correction2)[, adamw_decay]); adamw_decay = 1 - lr * weight_decay selects AdamW.
        Queued on `stream` (default: torch's current stream)."""
        import torch

        hp = _adam_hp(hp)
        h = (ctypes.c_float * 7)(*hp)
        pp, gp, st = ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(g.data_ptr()), self._stream_handle(stream)
        if p.dtype == torch.bfloat16:
            if w_off is None or g.dtype != torch.bfloat16:
                raise ValueError("bf16 parameters need bf16 gradients and w_off (fp32 master weights)")
            rc = self._c.lib.ocm_x_adam_bf16(self.handle, pp, gp, p.numel(), w_off, m_off, v_off, h, st)
        elif p.dtype == torch.float32 and g.dtype == torch.float32:
            rc = self._c.lib.ocm_x_adam(self.handle, pp, gp, p.numel(), m_off, v_off, h, st)
        else:
            raise ValueError(f"unsupported dtypes {p.dtype} / {g.dtype}")
        if rc != 0:
            raise OcmError("ocm_x_adam: " + last_error())

    def adam_multi(self, ps, gs, m_offs, v_offs, hp, w_offs=None, stream=None) -> None:
        """ocm_x_adam_multi: the fused update of many parameters, 32 per launch. ps / gs are
        lists of contiguous GPU tensors (all float32, or all bfloat16 with w_offs)."""
        import torch

        k = len(ps)
        bf16 = k > 0 and ps[0].dtype == torch.bfloat16
        if bf16 and w_offs is None:
            raise ValueError("bf16 parameters need w_offs (fp32 master weights)")
        arr_v, arr_u = ctypes.c_void_p * k, ctypes.c_uint64 * k
        hp = _adam_hp(hp)
        rc = self._c.lib.ocm_x_adam_multi(
            self.handle, k, arr_v(*[t.data_ptr() for t in ps]), arr_v(*[t.data_ptr() for t in gs]),
            arr_u(*[t.numel() for t in ps]), arr_u(*(w_offs or [0] * k)), arr_u(*m_offs), arr_u(*v_offs),
            (ctypes.c_float * 7)(*hp), 1 if bf16 else 0, self._stream_handle(stream))
        if rc != 0:
            raise OcmError("ocm_x_adam_multi: " + last_error())

    def time_onesided(self, op_flag: int, nbytes: int, iters: int, local_offset: int = 0, remote_offset: int = 0) -> float:
        """Seconds per blocking one-sided op, timed inside the native library."""
        p = OcmParams(local_offset, remote_offset, 0, 0, nbytes, op_flag)
        t = self._c.lib.ocm_x_time_onesided(self.handle, ctypes.byref(p), iters)
        if t < 0:
            raise OcmError("one-sided op failed: " + last_error())
        return t

    def time_onesided_samples(self, op_flag: int, nbytes: int, iters: int, gap_s: float = 0.0,
                              cap_s: float = 1.0, min_iters: int = 5, local_offset: int = 0,
                              remote_offset: int = 0) -> tuple[list, int]:
        """Seconds of each blocking one-sided op, timed one by one inside the native
        library: up to `iters` ops, stopping after `cap_s` (but not before `min_iters`),
        each after `gap_s` of busy host time that does not touch the library. Returns
        (samples, copy-service relaunches during the run)."""
        p = OcmParams(local_offset, remote_offset, 0, 0, nbytes, op_flag)
        out = (ctypes.c_double * max(1, iters))()
        rel = ctypes.c_uint64(0)
        n = self._c.lib.ocm_x_time_onesided_samples(self.handle, ctypes.byref(p), iters, min_iters,
                                                    int(gap_s * 1e9), int(cap_s * 1e9), out, ctypes.byref(rel))
        if n < 0:
            raise OcmError("one-sided op failed: " + last_error())
        return list(out[:n]), int(rel.value)

    def copy_in(self, src_ptr: int) -> None:
        if self._c.lib.ocm_copy_in(self.handle, ctypes.c_void_p(src_ptr)) != 0:
            raise OcmError("ocm_copy_in: " + last_error())

    def copy_out(self, dst_ptr: int) -> None:
        if self._c.lib.ocm_copy_out(ctypes.c_void_p(dst_ptr), self.handle) != 0:
            raise OcmError("ocm_copy_out: " + last_error())

    def fill(self, seed: int, offset: int = 0, nbytes: Optional[int] = None) -> None:
        """Write the deterministic word pattern into the local half."""
        ptr, n = self.localbuf()
        nbytes = n - offset if nbytes is None else nbytes
        if self._c.lib.ocm_x_pattern(ctypes.c_void_p(ptr + offset), nbytes // 4, offset // 4, seed, 0) != 0:
            raise OcmError("pattern fill failed")

    def check(self, seed: int, offset: int = 0, nbytes: Optional[int] = None, first_word: Optional[int] = None) -> int:
        """Mismatching 32-bit words of the local half against the pattern."""
        ptr, n = self.localbuf()
        nbytes = n - offset if nbytes is None else nbytes
        fw = offset // 4 if first_word is None else first_word
        bad = self._c.lib.ocm_x_pattern(ctypes.c_void_p(ptr + offset), nbytes // 4, fw, seed, 1)
        if bad < 0:
            raise OcmError("pattern check failed")
        return int(bad)

    # --- zero-copy torch views ---
    def _view(self, ptr: int, nbytes: int, dtype, on_device: bool):
        import torch

        class _Iface:  # __cuda_array_interface__ v3 (torch consumes it on ROCm too)
            def __init__(self, p, n):
                self.__cuda_array_interface__ = {"shape": (n,), "typestr": "|u1", "data": (p, False), "version": 3,
                                                 "strides": None, "stream": None}

        if on_device:
            t = torch.as_tensor(_Iface(ptr, nbytes), device=f"cuda:{self._c.device}")
        else:
            import ctypes as C

            buf = (C.c_uint8 * nbytes).from_address(ptr)
            t = torch.frombuffer(buf, dtype=torch.uint8)
        return t.view(dtype) if dtype is not None and dtype != torch.uint8 else t

    def local_tensor(self, dtype=None):
        """The local half as a tensor (on the app's GPU for GPU kinds, CPU otherwise). No copy."""
        ptr, n = self.localbuf()
        on_dev = self._c.device >= 0 and self.kind in (OCM_LOCAL_GPU, OCM_REMOTE_GPU)
        return self._view(ptr, n, dtype, on_dev)

    def remote_tensor(self, dtype=None):
        """The remote half (single extent) as a tensor on this process's GPU: torch kernels then
        read/write peer HBM directly over xGMI (or the pinned host tier over PCIe). No copy."""
        p = self._c.lib.ocm_remotebuf(self.handle)
        if not p:
            raise OcmError("remote_tensor needs a single-extent remote allocation")
        if self._c.device < 0:
            return self._view(p, self.remote_size(), dtype, False)
        return self._view(p, self.remote_size(), dtype, True)

    def free(self) -> None:
        if self.handle.value:
            rc = self._c.lib.ocm_free(self.handle)
            self.handle = ctypes.c_void_p(0)
            if rc != 0:
                raise OcmError("ocm_free: " + last_error())


def copy(dst: Allocation, src: Allocation, nbytes: int, src_offset: int = 0, dest_offset: int = 0,
         src_offset_2: int = 0, dest_offset_2: int = 0, op_flag: int = 1) -> None:
    """ocm_copy (two-sided, staged through the pair's local half; see oncillamem.h)."""
    p = OcmParams(src_offset, dest_offset, src_offset_2, dest_offset_2, nbytes, op_flag)
    if dst._c.lib.ocm_copy(dst.handle, src.handle, ctypes.byref(p)) != 0:
        raise OcmError("ocm_copy: " + last_error())


class Client:
    """Process attachment to the local ocmd (ocm_init / ocm_tini)."""

    def __init__(self, daemon_rank: Optional[int] = None, gpu: Optional[int] = None, ns: Optional[str] = None):
        if daemon_rank is not None:
            os.environ["OCM_DAEMON_RANK"] = str(daemon_rank)
        if gpu is not None:
            os.environ["OCM_GPU"] = str(gpu)
        if ns is not None:
            os.environ["OCM_NS"] = ns
        self.lib = load()
        self.open = False

    def __enter__(self) -> "Client":
        self.init()
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def init(self) -> None:
        if self.lib.ocm_init() != 0:
            raise OcmError("ocm_init: " + last_error())
        self.open = True

    def close(self) -> None:
        if self.open:
            self.lib.ocm_tini()
            self.open = False

    @property
    def rank(self) -> int:
        return int(self.lib.ocm_rank())

    @property
    def num_nodes(self) -> int:
        return int(self.lib.ocm_num_nodes())

    @property
    def device(self) -> int:
        return int(self.lib.ocm_device())

    def plan(self) -> Plan:
        """A new transfer plan (hipGraph replay of fixed batch schedules)."""
        return Plan(self)

    def alloc_latency(self, kind: int, samples: int, local_bytes: int = 0, remote_bytes: int = 0,
                      flags: int = 0) -> tuple:
        """Per-sample seconds of ocm_alloc_ex and the matching ocm_free, timed in C."""
        ap = OcmAllocParams(local_bytes, remote_bytes, kind)
        ex = OcmAllocExParams(-1, flags, 0, 0, 0)
        a = (ctypes.c_double * samples)()
        f = (ctypes.c_double * samples)()
        n = self.lib.ocm_x_alloc_latency(ctypes.byref(ap), ctypes.byref(ex), samples, a, f)
        if n != samples:
            raise OcmError(f"ocm_alloc/ocm_free failed after {n} samples: " + last_error())
        return list(a), list(f)

    def alloc(self, kind: int, local_bytes: int = 0, remote_bytes: int = 0, remote_rank: int = -1, flags: int = 0,
              stripe_width: int = 0, stripe_unit: int = 0) -> Allocation:
        ap = OcmAllocParams(local_bytes, remote_bytes, kind)
        if remote_rank < 0 and not flags and not stripe_width and not stripe_unit:
            h = self.lib.ocm_alloc(ctypes.byref(ap))
        else:
            ex = OcmAllocExParams(remote_rank, flags, stripe_width, 0, stripe_unit)
            h = self.lib.ocm_alloc_ex(ctypes.byref(ap), ctypes.byref(ex))
        if not h:
            raise OcmError("ocm_alloc: " + last_error())
        return Allocation(self, h, kind)

    def stats(self, rank: int = -1) -> dict:
        s = OcmDaemonStats()
        if self.lib.ocm_stats(rank, ctypes.byref(s)) != 0:
            raise OcmError("ocm_stats: " + last_error())
        return s.as_dict()
