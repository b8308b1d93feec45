"""Child process of tests/test_gpu_distributed.py::test_native_tiles_world_gt1_through_rccl_stub.

Runs the native row-tiled frame (csrc/rtx_tiles.hip) with world > 1 on the box's ONE GPU: every
rank of the frame is a host thread of this process with its own HipRenderer (workspace, learnt
order), its own HIP stream and its own plan, and the library's RCCL calls are bound to the
test-only stub (tests/stub_rccl.cpp, loaded by rtx_rccl_load(path) before anything else binds
RCCL: the binding is per process, hence the fresh child). The stub moves each matched send to its
receive with a device copy on the receiver's stream, in RCCL's pairwise posting order, so the
root's per-peer receives into recv + p * part_bytes, the peers' sends, gather_rows (RTX_TILES_ROWS)
and rtx_assemble_runs over unequal shares all run as they would over xGMI.

For every case the root's frames (two slots in flight: submit k, finish k - 1, as bench.py's tiles
mode) must equal a single-GPU render_tile of the same scene bit for bit, and the stub's call log
must show exactly the operations the plan's layout implies (peer, bytes, buffer addresses).
Prints one JSON line; exit status 0 only if every case passed.
"""

from __future__ import annotations

import ctypes
import json
import sys
import threading
import traceback
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

import torch  # noqa: E402

from python_ray_tracer_amd import scenes, tiling  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip import HipRenderer  # noqa: E402
from python_ray_tracer_amd.infrastructure.hip import _lib as L  # noqa: E402

STUB = (REPO / "tests" / "libstub_rccl.so").resolve()

# (name, world, (root_run, run), rows, out, scene spec, bounces, frames)
CASES = [
    ("n2_8to9_f32", 2, (8, 9), False, None, lambda: scenes.readme_spec(150, 97), 3, 4),
    ("n4_3to4_u8", 4, (3, 4), False, "u8", lambda: scenes.random_spec(16, 3, 160, 123), 4, 4),
    ("n8_1to2_u8", 8, (1, 2), False, "u8", lambda: scenes.random_spec(64, 5, 168, 203), 5, 4),
    ("n8_1to2_f32", 8, (1, 2), False, None, lambda: scenes.random_spec(64, 5, 168, 203), 5, 3),
    ("n4_rows_u8", 4, (1, 1), True, "u8", lambda: scenes.random_spec(16, 7, 136, 101), 3, 4),
    ("n3_3to4_f32_unbounded", 3, (3, 4), False, None, lambda: scenes.main_spec(120, 71), None, 3),
]


def stub_log(stub):
    n = stub.stub_rccl_log(None, 0)
    buf = (ctypes.c_longlong * (8 * max(n, 1)))()
    stub.stub_rccl_log(buf, n)
    keys = ("comm", "kind", "rank", "peer", "bytes", "ptr", "group", "seq")
    return [dict(zip(keys, buf[8 * i:8 * i + 8])) for i in range(n)]


def expected_ops(world, root_run, run, rows, W, H, rb, out, part_bytes, send_ptrs, recv_ptrs, frame_ptrs, n_frames):
    """The operations rtx_tiles_submit must post, per rank and frame (group): (kind, peer, bytes, ptr)."""
    ops = {}
    for r in range(world):
        for k in range(n_frames):
            slot = k % 2
            g = []
            if not rows:
                if r == 0:
                    g = [(1, p, part_bytes, recv_ptrs[slot] + p * part_bytes) for p in range(1, world)]
                else:
                    g = [(0, 0, part_bytes, send_ptrs[r][slot])]
            else:
                rowb = W * 3
                if r == 0:
                    for p in range(1, world):
                        n = tiling.n_local_rows(H, rb, world, p)
                        for j in range((n + rb - 1) // rb):
                            g.append((1, p, min(rb, n - j * rb) * rowb, frame_ptrs[k] + (j * world + p) * rb * rowb))
                else:
                    n = tiling.n_local_rows(H, rb, world, r)
                    g = [(0, 0, min(rb, n - j * rb) * rowb, send_ptrs[r][slot] + j * rb * rowb)
                         for j in range((n + rb - 1) // rb)]
            ops[(r, k)] = g
    return ops


def run_case(lib, stub, name, world, shares, rows, out, spec_fn, B, n_frames):
    dev = torch.device("cuda", 0)
    root_run, run = shares
    base = spec_fn()
    W, H = base["camera"]["width"], base["camera"]["height"]
    frames = [scenes.build_scene(scenes.with_camera(base, scenes.orbit_position(k, 11))) for k in range(n_frames)]
    ref = HipRenderer(max_bounces=B, color_dtype=torch.float32, device=dev)
    want = [ref.render_tile(sc, out=out).clone() for sc in frames]
    torch.cuda.synchronize()

    rb = 8
    dtype = torch.uint8 if out == "u8" else torch.float32
    item = torch.empty((), dtype=dtype).element_size()
    plen = tiling.part_len(H, W, rb, world, item, out, root_run, run)
    part_bytes = plen * item
    n_parts, shares_list = tiling.runs(world, root_run, run)
    kind = L.OUT_U8_HWC if out == "u8" else L.OUT_F32_SOA
    frame_shape = (H, W, 3) if out == "u8" else (3, H * W)

    uid = (ctypes.c_char * L.UNIQUE_ID_BYTES)()
    L.check(lib.rtx_comm_unique_id(uid), "rtx_comm_unique_id")
    stub.stub_rccl_reset()
    rends, plans, comms, sends, recvs, streams = [], [], [], [], [], []
    got = [torch.full(frame_shape, 7, dtype=dtype, device=dev) for _ in range(n_frames)]  # root frames
    for r in range(world):
        c = ctypes.c_void_p()
        L.check(lib.rtx_comm_init(uid, world, r, 0, ctypes.byref(c)), "rtx_comm_init")
        comms.append(c.value)
        rends.append(HipRenderer(max_bounces=B, color_dtype=torch.float32, device=dev))
        send = [torch.zeros(plen, dtype=dtype, device=dev) for _ in range(2)] if r != 0 else []
        recv = [torch.zeros((1 if rows else world, plen), dtype=dtype, device=dev) for _ in range(2)] if r == 0 else []
        sends.append(send)
        recvs.append(recv)
        ptrs = ctypes.c_void_p * 2
        plan = ctypes.c_void_p()
        L.check(lib.rtx_tiles_create(comms[r], world, r, 0, W, H, rb, kind, 2,
                                     ptrs(*[b.data_ptr() for b in send]) if send else None,
                                     ptrs(*[b.data_ptr() for b in recv]) if recv else None, part_bytes, root_run, run,
                                     (L.TILES_ROWS if rows else 0) | L.TILES_TIMED | (64 << L.F_RESERVE_SHIFT),
                                     ctypes.byref(plan)),
                f"rtx_tiles_create rank {r}")
        plans.append(plan.value)
        streams.append(torch.cuda.Stream(dev))
    torch.cuda.synchronize()

    errors = []

    def rank_main(r):
        try:
            first, my_run = shares_list[r]
            with torch.cuda.stream(streams[r]):
                h = L.stream_handle(streams[r])
                open_slot = None
                for k, sc in enumerate(frames):
                    slot = k % 2
                    rends[r].submit_tiles(plans[r], slot, sc, rb, n_parts, first, got[k] if r == 0 else None,
                                          part_run=my_run)
                    if open_slot is not None:
                        L.check(lib.rtx_tiles_finish(plans[r], open_slot, h), "rtx_tiles_finish")
                    open_slot = slot
                L.check(lib.rtx_tiles_finish(plans[r], open_slot, h), "rtx_tiles_finish")
            streams[r].synchronize()
        except Exception:  # noqa: BLE001 - reported by the main thread
            errors.append(f"rank {r}: {traceback.format_exc()[-1500:]}")

    threads = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=90)
    if any(t.is_alive() for t in threads):
        errors.append("a rank thread did not finish")
        return {"case": name, "ok": False, "errors": errors}
    torch.cuda.synchronize()

    res = {"case": name, "world": world, "shares": [root_run, run], "rows": rows, "out": out or "f32",
           "W": W, "H": H, "frames": n_frames, "part_bytes": part_bytes, "errors": errors}
    res["frames_equal"] = [bool(torch.equal(got[k], want[k])) for k in range(n_frames)]
    log = stub_log(stub)
    comm_ids = {rec["comm"] for rec in log}
    send_ptrs = {r: [b.data_ptr() for b in sends[r]] for r in range(1, world)}
    recv_ptrs = [b.data_ptr() for b in recvs[0]]
    want_ops = expected_ops(world, root_run, run, rows, W, H, rb, out, part_bytes, send_ptrs, recv_ptrs,
                            [g.data_ptr() for g in got], n_frames)
    got_ops = {}
    for rec in log:
        got_ops.setdefault((rec["rank"], rec["group"]), []).append((rec["kind"], rec["peer"], rec["bytes"], rec["ptr"]))
    res["log_ops"] = len(log)
    res["log_one_comm"] = len(comm_ids) == 1
    res["log_matches"] = got_ops == want_ops
    if not res["log_matches"]:
        bad = [k for k in sorted(set(want_ops) | set(got_ops)) if want_ops.get(k) != got_ops.get(k)][:3]
        res["log_diff"] = [(k, want_ops.get(k), got_ops.get(k)) for k in bad]
    res["stub_pending"] = stub.stub_rccl_pending()
    # RTX_TILES_TIMED: every rank's last gather span and the root's assembly (rtx_tiles_timing)
    timing = []
    for r in range(world):
        g, a = ctypes.c_float(), ctypes.c_float()
        L.check(lib.rtx_tiles_timing(plans[r], (n_frames - 1) % 2, ctypes.byref(g), ctypes.byref(a)),
                "rtx_tiles_timing")
        timing.append((round(g.value, 4), round(a.value, 4)))
    res["timing_ms"] = timing
    res["timing_ok"] = all(g >= 0 and a >= 0 for g, a in timing)
    for r in range(world):
        L.check(lib.rtx_tiles_destroy(plans[r]), "rtx_tiles_destroy")
        L.check(lib.rtx_comm_destroy(comms[r]), "rtx_comm_destroy")
    res["ok"] = (not errors and all(res["frames_equal"]) and res["log_matches"] and res["log_one_comm"]
                 and res["stub_pending"] == 0 and res["timing_ok"])
    return res


def main():
    assert torch.cuda.is_available(), "needs the GPU"
    torch.cuda.set_device(0)
    lib = L.load()
    stub = ctypes.CDLL(str(STUB))  # the same handle rtx_rccl_load's RTLD_NOLOAD dlopen returns
    stub.stub_rccl_log.argtypes = [ctypes.c_void_p, ctypes.c_int]
    stub.stub_rccl_set_timeout_ms(20000)
    L.check(lib.rtx_rccl_load(str(STUB).encode()), "rtx_rccl_load(stub)")
    only = set(sys.argv[1:])
    results = []
    for case in CASES:
        if only and case[0] not in only:
            continue
        try:
            results.append(run_case(lib, stub, *case))
        except Exception:  # noqa: BLE001
            results.append({"case": case[0], "ok": False, "errors": [traceback.format_exc()[-2000:]]})
        print(json.dumps(results[-1]), flush=True)
        if not results[-1]["ok"]:
            break  # (a failed case may leave operations unmatched: stop rather than time out the rest)
    ok = all(r["ok"] for r in results) and bool(results)
    print(json.dumps({"all_ok": ok, "cases": len(results)}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
