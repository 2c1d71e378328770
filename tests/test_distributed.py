"""Antenna sharding over ranks (world_size 2, gloo on CPU): the one-shot
setup collectives give every shard exactly what the unsharded run uses."""

import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ska_sdp_screen_fitting_amd.distributed import (check_distinct_devices,
                                                    gather_records, setup_shard,
                                                    shard_range)
from ska_sdp_screen_fitting_amd.geometry import piercepoints, grid_coords
from ska_sdp_screen_fitting_amd.stationscreen import station_orders
from ska_sdp_screen_fitting_amd.synthetic import (FIELD_DEC_DEG, FIELD_RA_DEG,
                                                  FIELD_WIDTH_DEG,
                                                  make_solutions)

N_TOTAL, T, F, D, CELL = 24, 3, 2, 12, 0.2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _slot_checksums(phi, w, st_order, pp, x, y, slots, ref_local=None):
    """Oracle fit + evaluation of sampled (t, f, a) slots of a [T, F, A, D]
    referenced block -> the sf_kl_eval_sums checksum of each slot's float32
    cube (sum mod 2^32 of its 32-bit words)."""
    from oracle import kl as okl
    basis = okl.Basis(pp)
    cpix = okl.cpix_matrix(pp, x, y)
    out = []
    for t, f, a in slots:
        if a == ref_local:  # the reference station keeps zero coefficients
            white = np.zeros(phi.shape[-1])
        else:
            white = okl.fit_slot(phi[t, f, a], w[t, f, a], st_order[a],
                                 st_order[a], basis)[0]
        planes = okl.eval_planes(okl.eval_phase_screens(white[None, :], cpix))
        words = planes.astype(np.float32).view(np.uint32).astype(np.uint64)
        out.append(int(words.sum() % 2 ** 32))
    return out


def _worker(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    a0, a1 = shard_range(N_TOTAL, world, rank)
    local = make_solutions(n_ant=a1 - a0, n_time=T, n_freq=F, n_dir=D,
                           ant_offset=a0, n_ant_total=N_TOTAL, flag_frac=0.05)
    st = setup_shard(local, a0, N_TOTAL, FIELD_RA_DEG, FIELD_DEC_DEG,
                     FIELD_WIDTH_DEG, CELL)
    # this shard's sampled slots, fitted and evaluated from the shard's own
    # setup (referenced with the broadcast reference phases)
    phi = local.val - st["ref_phase"].numpy()[:, :, None, :]
    slots = [(t, 0, a) for t in (0, T - 1) for a in (0, a1 - a0 - 1)]
    ref = st["ref_ant"]
    sums = _slot_checksums(phi, local.weight, st["st_order"], st["piercepoints"],
                           st["x"], st["y"], slots,
                           ref - a0 if a0 <= ref < a1 else None)
    np.savez(os.path.join(outdir, f"r{rank}.npz"), ref=st["ref_ant"],
             st_order=np.array(st["st_order"]), pp=st["piercepoints"],
             x=st["x"], y=st["y"], refph=st["ref_phase"].numpy(), a0=a0, a1=a1,
             slots=np.array(slots), sums=np.array(sums, np.uint64))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_covers_all():
    for n, w in ((256, 8), (10, 3), (7, 7), (5, 2)):
        ranges = [shard_range(n, w, r) for r in range(w)]
        assert ranges[0][0] == 0 and ranges[-1][1] == n
        assert all(ranges[i][1] == ranges[i + 1][0] for i in range(w - 1))


def test_shards_are_slices_of_the_full_set():
    full = make_solutions(n_ant=N_TOTAL, n_time=T, n_freq=F, n_dir=D)
    part = make_solutions(n_ant=8, n_time=T, n_freq=F, n_dir=D, ant_offset=8,
                          n_ant_total=N_TOTAL)
    np.testing.assert_array_equal(part.val, full.val[:, :, 8:16])
    np.testing.assert_array_equal(part.weight, full.weight[:, :, 8:16])
    np.testing.assert_array_equal(part.ant_pos, full.ant_pos[8:16])


@pytest.mark.timeout(300)
def test_setup_shard_world2_matches_unsharded(tmp_path):
    """Every rank's setup equals the unsharded run's, and the ORACLE's fit +
    evaluation of sampled slots from each shard's setup give the same cube
    checksums as the same slots of the unsharded setup (the GPU side of
    sharding: tests/test_slot_sums.py::test_sharded_gpu_sums_equal_unsharded
    and test_gpu_parity.py::test_fit_sharded_equals_unsharded)."""
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    full = make_solutions(n_ant=N_TOTAL, n_time=T, n_freq=F, n_dir=D,
                          flag_frac=0.05)
    w = np.sum(full.weight[:, :, :10], axis=(0, 1, 3), dtype=np.float64)
    ref = int(np.nonzero(w == w.max())[0][0])
    want_orders = station_orders(full.ant_pos, ref, min(20, D - 1))
    pp, mra, mdec = piercepoints(full.dir_radec)
    x, y = grid_coords(FIELD_RA_DEG, FIELD_DEC_DEG, FIELD_WIDTH_DEG, CELL, mra, mdec)
    got_orders = []
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        assert int(z["ref"]) == ref
        np.testing.assert_array_equal(z["pp"], pp)
        np.testing.assert_array_equal(z["x"], x)
        np.testing.assert_array_equal(z["y"], y)
        np.testing.assert_array_equal(z["refph"], full.val[:, :, ref, :])
        got_orders += list(z["st_order"])
        # the shard's sampled slots: the same cube checksums as the same
        # global slots of the unsharded run
        a0 = int(z["a0"])
        phi = full.val - full.val[:, :, ref:ref + 1, :]
        glob = [(t, f, a0 + a) for t, f, a in z["slots"]]
        want = _slot_checksums(phi, full.weight, want_orders, pp, x, y, glob, ref)
        assert [int(v) for v in z["sums"]] == want
    assert got_orders == want_orders


def _gather_worker(rank, world, port, outdir, same_card):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bus = 0x11 if same_card else 0x11 + rank
    ident = {"index": 0, "pci": f"0000:{bus:02x}:00", "uuid": f"GPU-{bus}",
             "rank": rank}
    idents = gather_records(ident)
    rec = gather_records({"rank": rank, "slots": 100 + rank, "eval_launch_ms": 1.5 * rank})
    try:
        check_distinct_devices(idents, "nccl")
        verdict = "ok"
    except RuntimeError as exc:
        verdict = str(exc)
    check_distinct_devices(idents, "gloo")  # rehearsals may share a card
    with open(os.path.join(outdir, f"g{rank}.json"), "w") as fh:
        json.dump([idents, rec, verdict], fh)
    dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("same_card", [False, True])
def test_rank_records_world2(tmp_path, same_card):
    """bench.py's ``dist`` object: every rank's device identity and numbers
    reach every rank in rank order; under nccl two ranks on one card are
    refused, under gloo allowed."""
    world = 2
    mp.start_processes(_gather_worker,
                       args=(world, _free_port(), str(tmp_path), same_card),
                       nprocs=world, join=True, start_method="spawn")
    for r in range(world):
        idents, rec, verdict = json.load(open(tmp_path / f"g{r}.json"))
        assert [d["rank"] for d in idents] == [0, 1]
        assert [d["slots"] for d in rec] == [100, 101]
        if same_card:
            assert "ranks 0 and 1 resolve to the same GPU" in verdict
        else:
            assert verdict == "ok"
