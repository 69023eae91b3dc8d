#!/usr/bin/env python3
"""Benchmark: MI355X FLAC frame decode on BASELINE config C2 (one JSON line on rank 0).

Workload: batches of 1024 synthetic frames (44.1 kHz / 16-bit stereo, blocksize 4096,
LPC order 8, Rice partition order 4), the compressed frames resident in HBM.  One step
decodes ``--batches`` independent batches (distinct copies in HBM, so nothing is served
from a previous step's cache footprint) into FLACDecoder's 16-bit interleaved LE PCM
(the OpenAL buffer-fill layout, FLACDecoder.cs:543-562) with the two kernels of the
path, k_parse and k_decode, on one HIP stream.

value      = decoded samples (blocksize x channels) per second,
             whole job over all ranks (weak scaling: every rank decodes its own batches).
roofline   = the dominant kernel (k_decode): algorithmic bytes (compressed frame bytes +
             PCM bytes written) / its HIP-event-timed average duration, vs 8 TB/s HBM.
cpu_baseline = the CPU restatement (oracle/: libFLAC 1.2.1 decode + FLACDecoder pack) on
             min(16, cpu count) threads, plus a 1-thread figure, on a bounded sample of
             the same frames.
Beside the metric (rank 0): indexer (bnflac_index_stream over one stream), reader
(bnflac_reader_* from host bytes to 16 KiB reads), pcie_inclusive (host-resident batches).

    python bench.py [--gpus N --steps K --warmup W --batches B]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded PCM MSamples/s/GPU (bit-exact) + achieved HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batches", type=int, default=1024,
                    help="C2 batches (x1024 frames) decoded per step; 128 = one k_decode_st wave (64 frames) "
                         "per resident slot (256 CUs x 8 waves); 1024 = eight such rounds (DESIGN.md section 5)")
    ap.add_argument("--frames", type=int, default=1024, help="frames per batch (BASELINE C2: 1024)")
    ap.add_argument("--groups", type=int, default=1,
                    help="pipeline groups: k_parse of group g+1 overlaps k_decode of group g (1 = serial)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline time budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads for the multi-thread CPU baseline (0: min(16, cpu count))")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive (host-resident) measurement")
    ap.add_argument("--no-index", action="store_true", help="skip the frame-indexer (bnflac_index_stream) timing")
    ap.add_argument("--no-reader", action="store_true", help="skip the streaming-reader (bnflac_reader_*) timing")
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    ap.add_argument("--stats", action="store_true", help="report k_decode event counters (one extra step)")
    ap.add_argument("--ablate", default=None,
                    help="comma list of ablation bitmasks to time after the measurement (timing only, wrong output): "
                         "1 CRC, 2 stores, 4 restore, 8 rice, 16 parse walk")
    return ap.parse_args()


def cpu_baseline(data: bytes, nsamples_per_pass: int, budget_s: float, threads: int = 1):
    """Oracle (restated libFLAC 1.2.1 + FLACDecoder.CopyTo pack) on `threads` host threads,
    each decoding whole batches independently (a libFLAC decoder is single-threaded per
    stream; ctypes releases the GIL during the call)."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.lib()
    counts = [0] * threads
    t0 = time.perf_counter()

    def run(i):
        while time.perf_counter() - t0 < budget_s:
            rc, pk, msg, _ = oracle.flacdecoder_copyto(data)
            assert rc == 0, msg
            counts[i] += 1

    ths = [threading.Thread(target=run, args=(i,)) for i in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    el = time.perf_counter() - t0
    passes = sum(counts)
    return passes * nsamples_per_pass / el / 1e6, passes, el


def measured_traffic(B: int, frames: int, G: int):
    """HBM bytes per k_decode launch from a committed PMC summary of this same workload
    (profiles/traffic_c2_b<B>.json, written from tools/pmc_session.sh counters with the
    MI355X_MICROARCH.md corrections).  PMC counters cannot be read from inside this run;
    None when no summary matches the configuration."""
    path = os.path.join(ROOT, "profiles", f"traffic_c2_b{B}.json")
    if G != 1 or not os.path.exists(path):
        return None
    d = json.load(open(path))
    if d.get("batches_per_step") != B or d.get("frames_per_batch") != frames:
        return None
    return {"traffic_bytes": int(d["traffic_bytes"]),
            "source": f"profiles/{os.path.basename(path)} ({d.get('round', '?')}: FETCH_SIZE x2 + WRITE_SIZE)"}


def cpu_model() -> str:
    try:
        for l in open("/proc/cpuinfo"):
            if l.startswith("model name"):
                return l.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def pcie_inclusive(args, torch, dev, libflac, dec, data, offs, sp, p, s, pcm_bytes, samples_per_batch, nb=8, reps=3):
    """Host-resident caller: pinned host compressed bytes -> H2D -> parse+decode -> D2H PCM.
    Reported beside `value`, never as it."""
    copy_len = (len(data) + 255) // 256 * 256
    h_in = torch.zeros(copy_len * nb + 64, dtype=torch.uint8).pin_memory()
    src = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy())
    for b in range(nb):
        h_in[b * copy_len: b * copy_len + len(data)] = src
    h_out = torch.empty(pcm_bytes * nb, dtype=torch.uint8).pin_memory()
    d_in = torch.empty_like(h_in, device=dev)
    d_out = torch.empty(pcm_bytes * nb, dtype=torch.uint8, device=dev)
    d_offs = torch.from_numpy(np.concatenate([offs + b * copy_len for b in range(nb)])).to(dev)
    fr_bs = np.full(args.frames, p.blocksize, dtype=np.int64)
    fr_start = np.concatenate([[0], np.cumsum(fr_bs)[:-1]])
    d_os = torch.from_numpy(np.concatenate([fr_start + b * int(s.nsamples) for b in range(nb)])).to(dev)
    nf = args.frames * nb
    d_info = torch.zeros(nf * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def once():
        d_in.copy_(h_in, non_blocking=True)
        dec.decode_frames(d_in, copy_len * nb, d_offs, nf, sp, libflac.OUT_FLACDECODER, d_out, d_info,
                          d_out_sample=d_os, stream=stream)
        h_out.copy_(d_out, non_blocking=True)

    once()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ok = h_out[:pcm_bytes].numpy().tobytes() == s.pcm.astype("<i2").tobytes()
    return {"value": round(samples_per_batch * nb * reps / el / 1e6, 2), "unit": "MSamples/s",
            "batches": nb * reps, "bitexact": bool(ok),
            "note": "pinned host bytes -> H2D -> k_parse+k_decode -> D2H PCM, serialized on one stream"}


def index_leg(torch, dev, libflac, dec, data, offs, sp, reps=5):
    """bnflac_index_stream over one whole C2 stream in HBM: sync scan,
    candidate parse, CRC-16 chain.  Wall time per call (it syncs once for the candidate
    count).  Reported beside `value`, not part of it."""
    n = len(data)
    d = torch.zeros((n + 15) // 16 * 16 + 16, dtype=torch.uint8, device=dev)
    d[:n] = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).to(dev)
    cap = len(offs) + 16
    o, _, _, nf = dec.index_stream(d, n, int(offs[0]), sp, cap)
    match = nf == len(offs) and bool(np.array_equal(o[:nf].cpu().numpy(), offs))
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        dec.index_stream(d, n, int(offs[0]), sp, cap)
    ms = (time.perf_counter() - t0) / reps * 1e3
    return {"ms": round(ms, 4), "GB_per_s": round(n / (ms * 1e-3) / 1e9, 2), "frames": nf, "stream_bytes": n,
            "matches_generator_offsets": match,
            "note": "one C2 stream: sync scan + k_parse of every candidate + CRC-16 chain (one host sync)"}


def reader_leg(libflac, data, pcm_ref: bytes, samples: int, reps=3, chunk=16384):
    """bnflac_reader over one whole C2 stream held in host memory: open
    (H2D, frame index, decode-ahead) + Read() in OpenAL-sized 16 KiB pieces until the end.
    Host-link and Python-call bound; reported beside `value`, not part of it."""
    best, ok = None, True
    for _ in range(reps):
        t0 = time.perf_counter()
        r = libflac.Reader(data, libflac.OUT_FLACDECODER)
        got = r.read_all(chunk)
        r.close()
        el = time.perf_counter() - t0
        ok = ok and got == pcm_ref
        best = el if best is None else min(best, el)
    return {"value": round(samples / best / 1e6, 2), "unit": "MSamples/s", "ms": round(best * 1e3, 2),
            "bitexact": bool(ok), "read_bytes": chunk,
            "note": "host bytes -> bnflac_reader_open (H2D, index, decode-ahead) -> Read() x 16 KiB until EOS"}


def main():
    args = parse_args()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    from birdnest.audio_amd import libflac, synth
    p = synth.config("C2", nframes=args.frames, seed=2)
    s = synth.encode(p)
    data = s.data.tobytes()
    offs = s.frame_offsets.astype(np.int64)
    fb_in = int(len(data) - offs[0])               # compressed frame bytes (sync .. CRC-16)
    samples_per_batch = int(s.nsamples) * p.channels
    sp = libflac.StreamParams.from_synth(p, s.nsamples)
    stride = libflac.out_stride(libflac.OUT_FLACDECODER, sp)
    pcm_bytes_per_batch = int(s.nsamples) * stride
    B = args.batches

    # B distinct copies of the batch in HBM (4-byte aligned), one output region each
    copy_len = (len(data) + 255) // 256 * 256
    one = np.zeros(copy_len, dtype=np.uint8)
    one[:len(data)] = np.frombuffer(data, dtype=np.uint8)
    d_bytes = torch.zeros(copy_len * B + 64, dtype=torch.uint8, device=dev)
    d_bytes[:copy_len * B].view(B, copy_len).copy_(torch.from_numpy(one).to(dev).unsqueeze(0).expand(B, copy_len))
    nbytes_total = copy_len * B
    d_offs = torch.from_numpy(np.concatenate([offs + b * copy_len for b in range(B)])).to(dev)
    nframes = args.frames * B
    fr_bs = np.full(args.frames, p.blocksize, dtype=np.int64)
    fr_start = np.concatenate([[0], np.cumsum(fr_bs)[:-1]])
    d_out_sample = torch.from_numpy(np.concatenate([fr_start + b * int(s.nsamples) for b in range(B)])).to(dev)
    d_out = torch.empty(pcm_bytes_per_batch * B, dtype=torch.uint8, device=dev)
    d_info = torch.zeros(nframes * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    dec = libflac.BatchDecoder(local_rank)
    stream = torch.cuda.current_stream(dev)

    # Pipelined schedule: B batches in G groups; k_parse of the next group (stream sP)
    # overlaps k_decode of the current one (stream sD).  Every timed step decodes all B
    # batches; the pipeline fill (first parse) is inside the timed region.
    G = args.groups
    if B % G:
        raise SystemExit("--batches must be a multiple of --groups")
    nf_g = nframes // G
    FIB = libflac.FRAME_INFO_BYTES
    sP = torch.cuda.Stream(dev)
    sD = torch.cuda.Stream(dev)
    ev_parsed = [torch.cuda.Event() for _ in range(G)]
    ev_decoded = [torch.cuda.Event() for _ in range(G)]
    views = [(d_offs[g * nf_g:(g + 1) * nf_g], d_out_sample[g * nf_g:(g + 1) * nf_g],
              d_info[g * nf_g * FIB:(g + 1) * nf_g * FIB]) for g in range(G)]

    def parse(g, tev=None):
        sP.wait_event(ev_decoded[g])  # the group's frame records are free again
        if tev is not None:
            tev[0].record(sP)
        o, osmp, inf = views[g]
        dec.parse_frames(d_bytes, nbytes_total, o, nf_g, sp, inf, d_out_sample=osmp, stream=sP)
        if tev is not None:
            tev[1].record(sP)
        ev_parsed[g].record(sP)

    def decode(g, tev=None):
        sD.wait_event(ev_parsed[g])
        if tev is not None:
            tev[0].record(sD)
        dec.decode_parsed(d_bytes, nbytes_total, nf_g, sp, libflac.OUT_FLACDECODER, d_out, views[g][2], stream=sD)
        if tev is not None:
            tev[1].record(sD)
        ev_decoded[g].record(sD)

    def run(K, pev=None, dev_=None):
        """K full steps; pev/dev_: per-launch timing event pairs (lists, appended to)."""
        def te(lst):
            if lst is None:
                return None
            e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            lst.append(e)
            return e
        parse(0, te(pev))
        for k in range(K):
            for g in range(G):
                decode(g, te(dev_))
                if g + 1 < G:
                    parse(g + 1, te(pev))
                elif k + 1 < K:
                    parse(0, te(pev))

    run(args.warmup)
    torch.cuda.synchronize(dev)
    pev, dev_ev = [], []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(args.steps, pev, dev_ev)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t_parse = sum(a.elapsed_time(b) for a, b in pev) / len(pev)  # ms per k_parse launch (one group)
    t_decode = sum(a.elapsed_time(b) for a, b in dev_ev) / len(dev_ev)  # ms per k_decode launch (one group)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    def step():  # one serial step on the default stream (stats / ablation timing)
        dec.parse_frames(d_bytes, nbytes_total, d_offs, nframes, sp, d_info, d_out_sample=d_out_sample, stream=stream)
        dec.decode_parsed(d_bytes, nbytes_total, nframes, sp, libflac.OUT_FLACDECODER, d_out, d_info, stream=stream)

    # correctness of what was timed: every frame ok, copies 0 and B-1 == source PCM
    info = libflac.info_array(d_info.view(-1, libflac.FRAME_INFO_BYTES)[:: max(1, nframes // 4096)].cpu().numpy())
    ok = bool((info["status"] == 0).all() and (info["crc_ok"] == 1).all())
    ref = s.pcm.astype("<i2").tobytes()
    for b in {0, B - 1}:
        got = d_out[b * pcm_bytes_per_batch:(b + 1) * pcm_bytes_per_batch].cpu().numpy().tobytes()
        ok = ok and got == ref
    if world > 1:
        o = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(o, op=dist.ReduceOp.MIN)
        ok = bool(o.item())

    total_samples = samples_per_batch * B * args.steps * world
    value = total_samples / elapsed / 1e6
    alg_bytes = (fb_in + pcm_bytes_per_batch) * (B // G)   # per k_decode launch (one group)
    achieved = alg_bytes / (t_decode * 1e-3) / 1e9
    step_achieved = alg_bytes * G / (elapsed / args.steps) / 1e9
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "MSamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic: deterministic generator (seed 2), BASELINE C2 frame shape",
        "config": {"workload": "C2: 1024-frame batches, 44.1 kHz/16-bit stereo, bs 4096, LPC-8, Rice partition "
                               "order 4 -> FLACDecoder 16-bit LE interleaved PCM",
                   "frames_per_batch": args.frames, "batches_per_step": B,
                   "compressed_bytes_per_batch": fb_in, "pcm_bytes_per_batch": pcm_bytes_per_batch,
                   "parallelism": f"frames sharded per rank x{world}",
                   "pipeline": (f"{G} groups of {B // G} batches: k_parse(g+1) || k_decode(g) on two streams"
                                if G > 1 else "serial: k_parse then k_decode over all batches")},
        "bitexact": ok,
        "roofline": {"bound": "hbm", "kernel": "k_decode", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": round(t_decode, 4),
                     "k_parse_avg_ms": round(t_parse, 4), "step_achieved_GBs": round(step_achieved, 1),
                     "launch": f"k_decode over one group ({B // G} batches x {args.frames} frames)"},
    }
    tr = measured_traffic(B, args.frames, G)
    if tr is not None:
        line["roofline"]["traffic"] = tr["traffic_bytes"]
        line["roofline"]["traffic_source"] = tr["source"]
    if args.stats and rank == 0:
        import ctypes
        buf = (ctypes.c_uint64 * 16)()
        dec.L.bnflac_debug_stats(buf, 1)
        dec.L.bnflac_debug_set_ablate(0x100)
        step()
        torch.cuda.synchronize(dev)
        dec.L.bnflac_debug_stats(buf, 1)
        dec.L.bnflac_debug_set_ablate(0)
        names = ["fused_chunks", "generic_chunks", "dma_land_waits", "slow_rice", "refills", "waves"]
        line["stats"] = {n: int(buf[i]) for i, n in enumerate(names)}
        w = max(1, int(buf[5]))
        line["stats"]["cycles_per_wave"] = {n: int(buf[8 + i]) // w for i, n in
                                            enumerate(["setup", "decode", "refill", "pack", "tail"])}
    if args.ablate and rank == 0:
        abl = []
        for m in [int(x, 0) for x in args.ablate.split(",")]:
            dec.L.bnflac_debug_set_ablate(m)
            run(1)
            pe, de = [], []
            run(args.steps, pe, de)
            torch.cuda.synchronize(dev)
            abl.append({"ablate": m, "k_parse_ms": round(sum(a.elapsed_time(b) for a, b in pe) / len(pe), 4),
                        "k_decode_ms": round(sum(a.elapsed_time(b) for a, b in de) / len(de), 4)})
        dec.L.bnflac_debug_set_ablate(0)
        line["ablation"] = abl
    if rank == 0 and not args.no_index:
        line["indexer"] = index_leg(torch, dev, libflac, dec, data, offs, sp)
    if rank == 0 and not args.no_reader:
        line["reader"] = reader_leg(libflac, data, s.pcm.astype("<i2").tobytes(), samples_per_batch)
    if rank == 0 and not args.no_pcie:
        line["pcie_inclusive"] = pcie_inclusive(args, torch, dev, libflac, dec, data, offs, sp, p, s,
                                                pcm_bytes_per_batch, samples_per_batch)
    if rank == 0 and not args.no_cpu_baseline:
        sys.stdout.flush()
        nthr = args.cpu_threads or min(16, os.cpu_count() or 1)
        mss1, passes1, el1 = cpu_baseline(data, samples_per_batch, args.cpu_seconds / 2, 1)
        mss, passes, el = cpu_baseline(data, samples_per_batch, args.cpu_seconds / 2, nthr)
        line["cpu_baseline"] = {"value": round(mss, 3), "unit": "MSamples/s", "cores": nthr, "kind": "port",
                                "sample": f"{passes} x one C2 batch ({args.frames} frames, {samples_per_batch} samples) "
                                          f"through the oracle's FLACDecoder.CopyTo replay on {nthr} threads, "
                                          f"{el:.1f} s",
                                "single_thread": {"value": round(mss1, 3), "cores": 1, "passes": passes1,
                                                  "seconds": round(el1, 2)},
                                "cpu": cpu_model()}
    if rank == 0:
        js = json.dumps(line)
        print(js, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(js + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
