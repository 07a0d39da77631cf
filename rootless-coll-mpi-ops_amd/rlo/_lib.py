"""ctypes binding of librlo_hip.so (include/rlo_hip.h).

The shared library is built in-tree (rootless-coll-mpi-ops_amd/lib/librlo_hip.so) by
`make -C rootless-coll-mpi-ops_amd` (or __graft_entry__.build()).  There is no CPU
fallback: if the library is missing the import fails loudly.
"""
import ctypes
import os
import re

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "lib", "librlo_hip.so")
# RLO_DIAG_LIB=1: the diagnostics build (make DIAG=1 -> lib_diag/), whose library honours the A/B
# environment switches the product library ignores (rlo_world.cpp diag_env).  RLO_LIB_DIR=lib_<name>: an
# A/B build in the package's lib_<name>/ (tools/ only)
if os.environ.get("RLO_DIAG_LIB") == "1":
    LIB_PATH = os.path.join(PKG_DIR, "lib_diag", "librlo_hip.so")
_AB = os.environ.get("RLO_LIB_DIR", "")
if re.fullmatch(r"lib_[a-z0-9_]+", _AB):
    LIB_PATH = os.path.join(PKG_DIR, _AB, "librlo_hip.so")

RLO_OK = 0
RLO_E_INVAL, RLO_E_HIP, RLO_E_OCCUPANCY, RLO_E_DEVICE, RLO_E_NOPROGRAM, RLO_E_NODEVICE = -1, -2, -3, -4, -5, -6
RLO_E_NOTCONNECTED = -7
RLO_E_AGAIN = -8
RLO_PART_BLOB_BYTES = 512
RLO_PART_UNCACHED = 1
RLO_PART_CHUNKED = 2
RLO_PART_PEND_HBM = 4
RLO_PART_ONE_XCD = 8
RLO_PEER_OTHER_GPU, RLO_PEER_IMPORTED = 1, 2  # rlo_world_info_t.peers
RLO_LAUNCH_NO_RESET = 1
RLO_TRIM_IMPORTS, RLO_TRIM_FREE, RLO_TRIM_RETIRED, RLO_TRIM_EXPORTED = 1, 2, 4, 8  # rlo_pool_trim
RLO_FLAG_LOG, RLO_FLAG_HIST, RLO_FLAG_PROF, RLO_FLAG_TIMELINE = 1, 2, 4, 8
RLO_JUDGE_APPROVE, RLO_JUDGE_MASK, RLO_JUDGE_ISP, RLO_JUDGE_HASH = 0, 1, 2, 3
DERR = {1: "timeout", 2: "vote ring", 3: "pid collision", 4: "vote orphan", 5: "log full", 6: "bad slot", 7: "host command",
        8: "bulk index"}
# host-service program (rlo_hip.h)
RLO_CMD_BCAST, RLO_CMD_PROPOSAL, RLO_CMD_JUDGE, RLO_CMD_OWN_JUDGE, RLO_CMD_QUIT = 0, 2, 16, 17, 18
RLO_CMD_BULK, RLO_CMD_BULK_RELEASE = 10, 19
RLO_EV_DELIVER_BCAST, RLO_EV_DELIVER_DECISION, RLO_EV_DELIVER_BULK = 1, 1 | (4 << 8), 1 | (10 << 8)
RLO_ORDER_RANDOM, RLO_ORDER_SLOTS = 0, 1
TAG_BULK = 10
RLO_EV_ACTION, RLO_EV_RESULT, RLO_EV_JUDGE, RLO_EV_OWN_JUDGE, RLO_EV_JUDGED = 3, 4, 6, 7, 8


class WorldCfg(ctypes.Structure):
    _fields_ = [("n_ranks", ctypes.c_int32), ("max_payload", ctypes.c_uint32), ("ring_slots", ctypes.c_uint32),
                ("device", ctypes.c_int32), ("bulk_max", ctypes.c_uint64), ("bulk_slots", ctypes.c_uint32),
                ("movers", ctypes.c_uint32), ("proposal_pool", ctypes.c_uint32), ("flags", ctypes.c_uint32)]


class WorldInfo(ctypes.Structure):
    _fields_ = [("n_ranks", ctypes.c_int32), ("max_in_degree", ctypes.c_int32), ("max_fanout", ctypes.c_int32),
                ("edges", ctypes.c_int32), ("ring_slots", ctypes.c_uint32), ("slot_stride", ctypes.c_uint32),
                ("vote_slots", ctypes.c_uint32), ("peers", ctypes.c_uint32), ("fwd_bytes", ctypes.c_uint64),
                ("vote_bytes", ctypes.c_uint64), ("ctrl_bytes", ctypes.c_uint64), ("cus", ctypes.c_int32),
                ("blocks_per_cu", ctypes.c_int32), ("part", ctypes.c_int32), ("n_parts", ctypes.c_int32),
                ("rank_begin", ctypes.c_int32), ("rank_end", ctypes.c_int32), ("sys_scope", ctypes.c_int32),
                ("waves", ctypes.c_int32), ("bulk_slots", ctypes.c_uint32), ("movers", ctypes.c_uint32),
                ("bulk_max", ctypes.c_uint64), ("heap_bytes", ctypes.c_uint64), ("proposal_pool", ctypes.c_uint32),
                ("pull", ctypes.c_uint32), ("nsmall", ctypes.c_uint32), ("stage2_bytes", ctypes.c_uint32),
                ("ll_ok", ctypes.c_uint32), ("pend_hbm", ctypes.c_uint32), ("dyn_lds", ctypes.c_uint32),
                ("static_lds", ctypes.c_uint32), ("last_kernel", ctypes.c_uint32), ("info_pad", ctypes.c_uint32)]


class PlanCfg(ctypes.Structure):
    _fields_ = [("n_ranks", ctypes.c_int32), ("n_parts", ctypes.c_int32), ("part", ctypes.c_int32),
                ("max_payload", ctypes.c_uint32), ("ring_slots", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("bulk_max", ctypes.c_uint64), ("bulk_slots", ctypes.c_uint32), ("movers", ctypes.c_uint32),
                ("proposal_pool", ctypes.c_uint32), ("cus", ctypes.c_int32)]


class PartCfg(ctypes.Structure):
    _fields_ = [("n_ranks", ctypes.c_int32), ("n_parts", ctypes.c_int32), ("part", ctypes.c_int32),
                ("part_begin", ctypes.c_void_p), ("max_payload", ctypes.c_uint32), ("ring_slots", ctypes.c_uint32),
                ("device", ctypes.c_int32), ("flags", ctypes.c_uint32), ("bulk_max", ctypes.c_uint64),
                ("bulk_slots", ctypes.c_uint32), ("movers", ctypes.c_uint32), ("proposal_pool", ctypes.c_uint32),
                ("pad", ctypes.c_uint32)]


class StormCfg(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("k", ctypes.c_int64), ("len", ctypes.c_uint32), ("window", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("log_cap", ctypes.c_uint32), ("len_max", ctypes.c_uint32),
                ("order", ctypes.c_uint32)]


class IarCfg(ctypes.Structure):
    _fields_ = [("judge_kind", ctypes.c_uint32), ("judge_ppm", ctypes.c_uint32), ("judge_seed", ctypes.c_uint64),
                ("judge_mask", ctypes.c_void_p), ("judge_isp", ctypes.c_char_p), ("flags", ctypes.c_uint32),
                ("log_cap", ctypes.c_uint32), ("pool", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


class HostCfg(ctypes.Structure):
    _fields_ = [("cmd_slots", ctypes.c_uint32), ("pickup_slots", ctypes.c_uint32), ("idle_timeout_s", ctypes.c_uint32),
                ("flags", ctypes.c_uint32), ("pool", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


class Cmd(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("origin", ctypes.c_int32), ("id", ctypes.c_int32), ("pseq", ctypes.c_uint32),
                ("vote", ctypes.c_int32), ("pad", ctypes.c_uint32)]


class RankStats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_uint64) for f in (
        "bcast_delivered", "bcast_sum", "originated", "dec_delivered", "dec_approved", "actions", "judge_calls",
        "own_decided", "own_approved", "proposals_recv", "iterations", "busy_iterations", "stalls", "log_count",
        "t_start", "t_end")] + [("error", ctypes.c_uint32), ("error_aux", ctypes.c_uint32), ("prof", ctypes.c_uint64 * 8),
                           ("dbg", ctypes.c_uint64 * 8),
                           ("hist", ctypes.c_uint32 * 128), ("unmarked_slots", ctypes.c_uint64)]


class BulkPlan(ctypes.Structure):
    _fields_ = [("nchunks", ctypes.c_uint32), ("stripe", ctypes.c_uint32), ("chunk", ctypes.c_uint32),
                ("tile", ctypes.c_uint32), ("total_tiles", ctypes.c_uint32), ("direct", ctypes.c_uint32)]


class LogRec(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("origin", ctypes.c_int32), ("from_", ctypes.c_int32), ("id", ctypes.c_uint32),
                ("len", ctypes.c_uint32), ("vote", ctypes.c_int32), ("aux", ctypes.c_uint32), ("payload_idx", ctypes.c_uint32)]


# every symbol include/rlo_hip.h declares (checked by tests/test_abi.py)
EXPORTS = ["rlo_topology", "rlo_children", "rlo_world_create", "rlo_world_destroy", "rlo_part_close_imports", "rlo_part_import", "rlo_world_query",
           "rlo_part_create", "rlo_part_export", "rlo_part_connect", "rlo_reset", "rlo_launch_ex",
           "rlo_stream_create", "rlo_stream_destroy",
           "rlo_program_storm", "rlo_program_latency", "rlo_program_iar", "rlo_launch", "rlo_wait", "rlo_run",
           "rlo_last_kernel_ms", "rlo_stats", "rlo_log", "rlo_latencies", "rlo_round_ticks", "rlo_timeline", "rlo_strerror", "rlo_last_hip_error",
           "rlo_device_error", "rlo_bulk_debug",
           "rlo_program_host", "rlo_host_post", "rlo_host_poll", "rlo_host_running", "rlo_host_cmd_count",
           "rlo_device_count", "rlo_device_numa_node", "rlo_host_bulk_stage", "rlo_host_bulk_copy", "rlo_bulk_plan", "rlo_layout_plan",
           "rlo_storm_lengths", "rlo_host_share", "rlo_host_unlink", "rlo_host_proxy", "rlo_host_wait_started",
           "rlo_host_fail", "rlo_client_attach", "rlo_client_detach", "rlo_client_state", "rlo_client_post",
           "rlo_client_poll", "rlo_client_cmd_count", "rlo_client_bulk_put", "rlo_client_bulk_get", "rlo_client_debug", "rlo_client_hdiag", "rlo_client_fwd", "rlo_host_device_judge",
           "rlo_pool_trim", "rlo_pool_stats"]

_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("librlo_hip.so not built (%s): run `make -C rootless-coll-mpi-ops_amd`" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    ip = ctypes.POINTER(ctypes.c_int)
    vp = ctypes.c_void_p
    L.rlo_topology.argtypes = [ctypes.c_int, ctypes.c_int, ip, ip, ip, ip, ip]
    L.rlo_children.argtypes = [ctypes.c_int] * 4 + [ip]
    L.rlo_world_create.argtypes = [ctypes.POINTER(WorldCfg), ctypes.POINTER(vp)]
    L.rlo_world_destroy.argtypes = [vp]
    L.rlo_part_close_imports.argtypes = [vp]
    L.rlo_pool_trim.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
    L.rlo_pool_stats.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
    L.rlo_part_import.argtypes = [vp, ctypes.c_char_p, ctypes.c_int]
    L.rlo_world_query.argtypes = [vp, ctypes.POINTER(WorldInfo)]
    L.rlo_program_storm.argtypes = [vp, ctypes.POINTER(StormCfg)]
    L.rlo_program_latency.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32]
    L.rlo_program_iar.argtypes = [vp, ctypes.POINTER(IarCfg), ctypes.c_int64, vp, vp, vp, vp, vp]
    L.rlo_part_create.argtypes = [ctypes.POINTER(PartCfg), ctypes.POINTER(vp)]
    L.rlo_part_export.argtypes = [vp, vp, ctypes.c_uint32]
    L.rlo_part_connect.argtypes = [vp, vp, ctypes.c_int]
    L.rlo_reset.argtypes = [vp, vp]
    L.rlo_launch_ex.argtypes = [vp, vp, ctypes.c_uint32]
    L.rlo_launch.argtypes = [vp, vp]
    L.rlo_stream_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.rlo_stream_destroy.argtypes = [vp]
    L.rlo_wait.argtypes = [vp]
    L.rlo_run.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_float)]
    L.rlo_last_kernel_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    L.rlo_stats.argtypes = [vp, ctypes.POINTER(RankStats), ctypes.c_int]
    L.rlo_log.argtypes = [vp, ctypes.c_int, ctypes.POINTER(LogRec), ctypes.c_uint32, vp, ctypes.c_uint32]
    L.rlo_latencies.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
    L.rlo_round_ticks.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
    L.rlo_timeline.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint32)]
    L.rlo_program_host.argtypes = [vp, ctypes.POINTER(HostCfg)]
    L.rlo_host_post.argtypes = [vp, ctypes.c_int, ctypes.POINTER(Cmd), vp, ctypes.c_uint32]
    L.rlo_host_poll.argtypes = [vp, ctypes.c_int, ctypes.POINTER(LogRec), vp, ctypes.c_uint32]
    L.rlo_host_running.argtypes = [vp]
    L.rlo_host_cmd_count.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    L.rlo_device_count.argtypes = []
    L.rlo_device_numa_node.argtypes = [ctypes.c_int]
    L.rlo_host_bulk_stage.argtypes = [vp, ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_uint32,
                                      ctypes.POINTER(ctypes.c_uint32)]
    L.rlo_host_bulk_copy.argtypes = [vp, ctypes.c_int, ctypes.POINTER(LogRec), vp]
    L.rlo_bulk_plan.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(BulkPlan)]
    L.rlo_layout_plan.argtypes = [ctypes.POINTER(PlanCfg), ctypes.POINTER(WorldInfo)]
    L.rlo_storm_lengths.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.POINTER(ctypes.c_uint32)]
    L.rlo_host_device_judge.argtypes = [vp, ctypes.POINTER(IarCfg)]
    L.rlo_host_share.argtypes = [vp, ctypes.c_char_p, ctypes.c_uint64]
    L.rlo_host_unlink.argtypes = [vp]
    L.rlo_host_proxy.argtypes = [vp]
    L.rlo_host_wait_started.argtypes = [vp, ctypes.c_uint32]
    L.rlo_host_fail.argtypes = [vp]
    L.rlo_client_attach.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(vp)]
    L.rlo_client_detach.argtypes = [vp]
    L.rlo_client_state.argtypes = [vp]
    L.rlo_client_post.argtypes = [vp, ctypes.POINTER(Cmd), vp, ctypes.c_uint32]
    L.rlo_client_poll.argtypes = [vp, ctypes.POINTER(LogRec), vp, ctypes.c_uint32]
    L.rlo_client_cmd_count.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    L.rlo_client_bulk_put.argtypes = [vp, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    L.rlo_client_bulk_get.argtypes = [vp, ctypes.POINTER(LogRec), vp]
    L.rlo_client_debug.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    L.rlo_client_hdiag.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    L.rlo_client_fwd.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_int64)]
    L.rlo_bulk_debug.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
    L.rlo_device_error.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    L.rlo_strerror.argtypes = [ctypes.c_int]
    L.rlo_strerror.restype = ctypes.c_char_p
    _lib = L
    return L


class RloError(RuntimeError):
    pass


def check(rc, what=""):
    if rc < 0:
        L = load()
        msg = L.rlo_strerror(rc).decode()
        if rc == RLO_E_HIP:
            msg += " (hipError %d)" % L.rlo_last_hip_error()
        raise RloError("%s failed: %s [%d]" % (what, msg, rc))
    return rc
