#!/usr/bin/env python3
"""Benchmark: MI355X FLAC frame decode on the BASELINE.json configs (one JSON line on rank 0).

Headline (`--config C2`, the default): batches of 1024 synthetic frames (44.1 kHz / 16-bit
stereo, blocksize 4096, LPC order 8, Rice partition order 4), compressed frames resident in
HBM.  One step decodes ``--batches`` independent copies (distinct HBM regions, so nothing is
served from a previous step's cache footprint) into FLACDecoder's 16-bit interleaved LE PCM
(the OpenAL buffer-fill layout, FLACDecoder.cs:543-562) with the two launches of the path,
k_parse and the decode launch, on one HIP stream.  The decode launch picks its kernels from the
parse's frame classes: k_decode_st (stereo LPC <= 8, C2), k_decode_sw (24-bit stereo, C3),
k_decode<8|16|32> (the rest), or k_decode_sys (the systolic LPC restore) for launches too small
to fill the chip with one subframe per lane (C5, the reader).

The other 1-GPU configs are side legs of the same line (rank 0, N = 1 only; `--legs`):
  C3  96 kHz/24-bit stereo, LPC-12, bs 8192, wasted bits + mid/side -> FLACFileReader 3-byte PCM
  C4  mixed CONSTANT/VERBATIM/FIXED/LPC, variable bs 192-16384, 16-bit stereo -> FLACDecoder PCM
  C5  8 distinct 192 kHz/24-bit 8-channel LPC-32 files (469 frames each, c5_job at one rank)
      -> FLACFileReader 3-byte PCM
Each leg reports value, the decode launch's roofline, a step-level roofline and its own
cpu_baseline.  `--config C5` makes C5 the headline: 8 files sharded over the ranks
(shard.partition), each rank indexing its files on the GPU (bnflac_index_stream) and decoding
them, then the interleaved PCM gathered to rank 0 over RCCL (shard.gather_bytes, concurrent
point-to-point receives); decode-only and decode+gather times are reported separately.

value        = decoded samples (blocksize x channels) per second, whole
               job over all ranks (weak scaling for C2-C4: a corpus of N x B batches, rank r decoding
               its contiguous B of them, a stream of its own).
roofline     = the dominant launch (the decode launch): algorithmic bytes (compressed frame bytes +
               PCM bytes written) / its HIP-event-timed average duration on the stream it
               runs on, vs 8 TB/s HBM; step_frac = the same bytes / the whole step (k_parse included).
cpu_baseline = the CPU restatement (oracle/: libFLAC 1.2.1 decode + the C# pack of the config) on
               every host core this process may use (os.sched_getaffinity), plus a 1-thread figure,
               on a bounded sample of the same frames.

    python bench.py [--gpus N --steps K --warmup W --batches B --config C2|C3|C4|C5 --legs C3,C4,C5]
    torchrun --nproc-per-node N bench.py --gpus N ...   (or: python bench.py --gpus N, which starts the
                                                         N rank processes itself)
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded PCM MSamples/s/GPU (bit-exact) + achieved HBM GB/s vs roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

# per config: output layout of the reference's C# surface for it, default copies per step,
# and what the config is (BASELINE.json configs[1..4])
CONFIGS = {
    "C2": dict(fmt="FLACDECODER", batches=1024, frames=1024,
               desc="C2: 1024-frame batches, 44.1 kHz/16-bit stereo, bs 4096, LPC-8, Rice partition order 4 "
                    "-> FLACDecoder 16-bit LE interleaved PCM"),
    # C3/C4: 256 copies per step.  A C4 frame of 16384 samples is one lane's serial work, so
    # at 32 copies the decode launch is as long as 1 copy (31.6 ms either way, r2 sweep):
    # the step must hold enough frames to fill the chip (C4 256: 10.5 GB compressed, below
    # the 16 GiB per-call limit)
    "C3": dict(fmt="FILEREADER", batches=256, frames=1024,
               desc="C3: 1024-frame batches, 96 kHz/24-bit stereo, LPC-12, bs 8192, wasted bits + mid/side "
                    "-> FLACFileReader 24-bit LE interleaved PCM"),
    "C4": dict(fmt="FLACDECODER", batches=256, frames=4096,
               desc="C4: 4096-frame mixed corpus (CONSTANT/VERBATIM/FIXED/LPC, variable bs 192-16384), "
                    "16-bit stereo -> FLACDecoder 16-bit LE interleaved PCM"),
    "C5": dict(fmt="FILEREADER", batches=8, frames=469,
               desc="C5: 10 s files, 192 kHz/24-bit 8-channel, LPC-32, bs 4096 -> FLACFileReader 24-bit LE "
                    "interleaved PCM"),
}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); without a launcher (WORLD_SIZE unset) bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS), help="headline workload")
    ap.add_argument("--batches", type=int, default=0,
                    help="copies decoded per step (0: the config's default; C2: 1024 = eight rounds of "
                         "k_decode_st waves, DESIGN.md section 5; C5: files in the job)")
    ap.add_argument("--frames", type=int, default=0, help="frames per batch (0: the config's)")
    ap.add_argument("--legs", default="C3,C4,C5", help="side legs at N = 1 (comma list, '' for none)")
    ap.add_argument("--leg-steps", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline time budget (headline)")
    ap.add_argument("--leg-cpu-seconds", type=float, default=3.0, help="CPU baseline time budget per leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="host threads for the multi-thread CPU baseline (0: every core in the affinity mask)")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive (host-resident) measurement")
    ap.add_argument("--no-index", action="store_true", help="skip the frame-indexer (bnflac_index_stream) timing")
    ap.add_argument("--no-reader", action="store_true", help="skip the streaming-reader (bnflac_reader_*) timing")
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    ap.add_argument("--nccl-timeout", type=int, default=180, help="seconds before a stuck collective aborts the run")
    ap.add_argument("--no-c5-flow", action="store_true",
                    help="N > 1: skip the C5 shard -> index -> decode -> RCCL gather leg")
    ap.add_argument("--c5-split", type=int, default=1,
                    help="C5 flow at N > 1: the in-step gather's groups are K frame ranges of each file "
                         "(default 1: whole files; one file's decode is latency-bound, so K pieces decode "
                         "in about K times its time)")
    ap.add_argument("--c5-batch", action="store_true",
                    help="--config C5 as one batch of the 8 files' frames (the C5 leg's workload; --stats/--ablate apply)")
    ap.add_argument("--stats", action="store_true", help="report k_decode event counters (one extra step)")
    ap.add_argument("--ablate", default=None,
                    help="comma list of ablation bitmasks to time after the measurement (timing only, wrong output): "
                         "1 CRC, 2 stores, 4 restore, 8 rice, 16 parse walk")
    ap.add_argument("--spawn-dry-run", action="store_true", help=argparse.SUPPRESS)  # print the rank plan (tests)
    ap.add_argument("--rank-selftest", action="store_true", help=argparse.SUPPRESS)  # gloo all_reduce per rank (tests)
    return ap.parse_args()


# --------------------------------------------------------------------------- rank launcher
def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_plan(n: int, port: int) -> list:
    """The environment of each of n rank processes on this node (torch.distributed.run's
    variables; rendezvous on 127.0.0.1)."""
    return [{"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
             "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)} for r in range(n)]


def launch_ranks(args) -> int | None:
    """`--gpus N` and the process count must agree.  Under a launcher (WORLD_SIZE set) a
    mismatch is refused; without one, N > 1 starts the N rank processes here -- children, not
    an exec, and before anything in this process touches the GPU -- and returns their exit
    status (the first failure ends the others, so a dead rank cannot leave its peers waiting in
    a collective).  None: this process is a rank (or the only one) and runs the bench."""
    world_env = os.environ.get("WORLD_SIZE") or None
    if world_env is not None:
        if args.gpus is not None and int(world_env) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}: refusing a mismatched run",
                  file=sys.stderr, flush=True)
            return 2
        return None
    n = args.gpus or 1
    if n <= 1:
        return None
    plan = rank_plan(n, _free_port())
    if args.spawn_dry_run:
        print(json.dumps({"ranks": plan, "argv": sys.argv[1:]}), flush=True)
        return 0
    import subprocess
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=dict(os.environ, **e))
             for e in plan]
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:  # the exact children this launcher started
                    q.terminate()
        time.sleep(0.05)
    return rc


def rank_selftest(args) -> None:
    """One gloo all_reduce per rank (CPU): proves the launcher's rank environment."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    t = torch.tensor([rank + 1], dtype=torch.int64)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"world": world, "sum": int(t.item()), "gpus": args.gpus,
                          "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def affinity_cores() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def host_threads() -> int:
    """Every core this process may use, capped by the box's CPU share for one GPU when the
    environment states one (OMP_NUM_THREADS: the GPU box sets it to its share)."""
    n = affinity_cores()
    share = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(share)) if share.isdigit() and int(share) > 0 else n


def cpu_model() -> str:
    try:
        for l in open("/proc/cpuinfo"):
            if l.startswith("model name"):
                return l.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def kernels_sha() -> str:
    """Hash of every source, header and hipcc flag the timed library was built from
    (build.source_hash; ties a committed PMC traffic summary to this build)."""
    from birdnest.audio_amd import build
    return build.source_hash()


def pack_reference(pcm: np.ndarray, fmt: str, bps: int) -> bytes:
    """Expected bytes of the lossless round trip in the C# layout (generator PCM is the golden)."""
    if fmt == "FLACDECODER":
        return pcm.astype("<i2").tobytes()
    if bps == 16:
        return pcm.astype("<i2").tobytes()
    return np.ascontiguousarray(pcm.astype("<i4")).view(np.uint8).reshape(-1, 4)[:, :3].tobytes()


class Workload:
    """B copies of one synthetic stream's frames resident in HBM, with their records and output."""

    def __init__(self, cfg, B, frames, torch, dev, libflac, synth, dec, seed=None):
        c = CONFIGS[cfg]
        self.cfg, self.B = cfg, B
        kw = {"nframes": frames or c["frames"]}
        if seed is not None:
            kw["seed"] = seed
        p = synth.config(cfg, **kw)
        if kw["nframes"] != CONFIGS[cfg]["frames"] and p.last_blocksize:
            p.last_blocksize = 0
        s = synth.encode(p)
        self.p, self.s = p, s
        self.data = s.data.tobytes()
        self.offs = s.frame_offsets.astype(np.int64)
        self.nf1 = len(self.offs)
        self.fb_in = int(len(self.data) - self.offs[0])          # compressed frame bytes (sync .. CRC-16)
        self.samples1 = int(s.nsamples) * p.channels
        self.fmt_name = c["fmt"]
        self.fmt = getattr(libflac, "OUT_" + c["fmt"])
        self.sp = libflac.StreamParams.from_synth(p, s.nsamples)
        self.stride = libflac.out_stride(self.fmt, self.sp)
        self.pcm1 = int(s.nsamples) * self.stride
        self.ref = pack_reference(s.pcm, c["fmt"], p.bps)
        assert len(self.ref) == self.pcm1
        self.torch, self.dev, self.libflac, self.dec = torch, dev, libflac, dec
        copy_len = (len(self.data) + 255) // 256 * 256
        self.copy_len = copy_len
        one = np.zeros(copy_len, dtype=np.uint8)
        one[:len(self.data)] = np.frombuffer(self.data, dtype=np.uint8)
        self.d_bytes = torch.zeros(copy_len * B + 64, dtype=torch.uint8, device=dev)
        self.d_bytes[:copy_len * B].view(B, copy_len).copy_(torch.from_numpy(one).to(dev).unsqueeze(0).expand(B, copy_len))
        self.nbytes = copy_len * B
        # frame positions of copy 0 from the headers (variable blocksizes: sample numbers)
        d_o1 = torch.from_numpy(self.offs).to(dev)
        d_i1 = torch.zeros(self.nf1 * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
        dec.parse_frames(self.d_bytes, copy_len, d_o1, self.nf1, self.sp, d_i1)
        torch.cuda.synchronize(dev)
        inf = libflac.info_array(d_i1.cpu().numpy())
        assert (inf["status"] == 0).all(), "k_parse rejected a generated frame"
        fr_start = inf["out_sample"].astype(np.int64)
        self.nframes = self.nf1 * B
        self.d_offs = torch.from_numpy(np.concatenate([self.offs + b * copy_len for b in range(B)])).to(dev)
        self.d_os = torch.from_numpy(np.concatenate([fr_start + b * int(s.nsamples) for b in range(B)])).to(dev)
        self.d_out = torch.empty(self.pcm1 * B, dtype=torch.uint8, device=dev)
        self.d_info = torch.zeros(self.nframes * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
        self.alg_bytes = (self.fb_in + self.pcm1) * B       # per decode launch
        self.samples = self.samples1 * B                     # per step

    def parse(self, stream):
        self.dec.parse_frames(self.d_bytes, self.nbytes, self.d_offs, self.nframes, self.sp, self.d_info,
                              d_out_sample=self.d_os, stream=stream)

    def decode(self, stream):
        self.dec.decode_parsed(self.d_bytes, self.nbytes, self.nframes, self.sp, self.fmt, self.d_out, self.d_info,
                               stream=stream)

    def run(self, K, stream, pev=None, dev_ev=None):
        torch = self.torch
        for _ in range(K):
            if pev is not None:
                e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                e[0].record(stream)
                self.parse(stream)
                e[1].record(stream)
                pev.append(e)
            else:
                self.parse(stream)
            if dev_ev is not None:
                e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                e[0].record(stream)
                self.decode(stream)
                e[1].record(stream)
                dev_ev.append(e)
            else:
                self.decode(stream)

    def check(self) -> bool:
        """Every frame record of every copy OK with its CRC-16 checked, copy 0's PCM equal to the
        source PCM, and every other copy's PCM equal to copy 0's (compared on the device, in
        chunks of copies: all B copies decode the same bytes)."""
        lf, torch = self.libflac, self.torch
        info = lf.info_array(self.d_info.cpu().numpy())
        ok = bool(len(info) == self.nframes and (info["status"] == 0).all() and (info["crc_ok"] == 1).all())
        v = self.d_out[:self.pcm1 * self.B].view(self.B, self.pcm1)
        ok = ok and v[0].cpu().numpy().tobytes() == self.ref
        step = max(1, (1 << 29) // self.pcm1)
        for b in range(1, self.B, step):
            e = min(self.B, b + step)
            ok = ok and bool(torch.equal(v[b:e], v[0:1].expand(e - b, self.pcm1)))
        return ok


def timed(wl, steps, warmup, stream, world, dist, dev):
    """warmup, then K timed steps between barriers + device syncs; returns elapsed (max over
    ranks), k_parse and decode-launch averages (ms, HIP events on the launch stream)."""
    torch = wl.torch
    wl.run(warmup, stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    pev, dev_ev = [], []
    t0 = time.perf_counter()
    wl.run(steps, stream, pev, dev_ev)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t_parse = sum(a.elapsed_time(b) for a, b in pev) / len(pev)
    t_decode = sum(a.elapsed_time(b) for a, b in dev_ev) / len(dev_ev)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, t_parse, t_decode


def roofline(alg_bytes, t_decode_ms, t_parse_ms, step_ms, traffic=None):
    achieved = alg_bytes / (t_decode_ms * 1e-3) / 1e9
    step = alg_bytes / (step_ms * 1e-3) / 1e9
    r = {"bound": "hbm", "kernel": "decode launch (frame order + k_decode_st + k_decode<8|16|32>)",
         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
         "traffic": None, "alg_bytes_per_launch": int(alg_bytes), "avg_launch_ms": round(t_decode_ms, 4),
         "k_parse_avg_ms": round(t_parse_ms, 4), "step_achieved_GBs": round(step, 1),
         "step_frac": round(step / HBM_PEAK_GBS, 4)}
    if traffic is not None:
        r["traffic"] = traffic["traffic_bytes"]
        r["traffic_over_alg"] = round(traffic["traffic_bytes"] / alg_bytes, 3)
        r["traffic_source"] = traffic["source"]
    return r


def measured_traffic(cfg: str, B: int, frames: int):
    """HBM bytes per decode launch from a committed PMC summary of this workload AND this build
    (profiles/traffic_<cfg>_b<B>.json from tools/pmc_session.sh + tools/pmc_summary.py, with the
    MI355X_MICROARCH.md FETCH_SIZE correction).  Counters cannot be read inside the timed run;
    None when no summary matches the workload and the kernel sources' hash."""
    path = os.path.join(ROOT, "profiles", f"traffic_{cfg.lower()}_b{B}.json")
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    if d.get("batches_per_step") != B or d.get("frames_per_batch") != frames or d.get("kernels_sha") != kernels_sha():
        return None
    return {"traffic_bytes": int(d["traffic_bytes"]),
            "source": f"profiles/{os.path.basename(path)} ({d.get('round', '?')}, kernels {d['kernels_sha']}: "
                      f"FETCH_SIZE x2 + WRITE_SIZE)"}


# --------------------------------------------------------------------------- CPU baseline
def cpu_baseline(data: bytes, fmt: str, buf_len: int, samples_per_pass: int, budget_s: float, threads: int):
    """The oracle (restated libFLAC 1.2.1 + the C# pack of the layout) on `threads` host threads,
    each decoding whole streams independently (a libFLAC decoder is single-threaded per stream;
    ctypes releases the GIL during the call)."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.lib()
    counts = [0] * threads
    t0 = time.perf_counter()

    def run(i):
        while time.perf_counter() - t0 < budget_s:
            if fmt == "FLACDECODER":
                rc, _, msg, _ = oracle.flacdecoder_copyto(data)
            else:
                rc, _, msg = oracle.filereader_readall(data, buf_len=buf_len)
            assert rc == 0, msg
            counts[i] += 1

    ths = [threading.Thread(target=run, args=(i,)) for i in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    el = time.perf_counter() - t0
    passes = sum(counts)
    return passes * samples_per_pass / el / 1e6, passes, el


def cpu_leg(wl, budget_s, threads_arg):
    nthr = threads_arg or host_threads()
    p = wl.p
    buf_len = p.blocksize * p.channels * (3 if p.bps == 24 else 2)  # one frame per FLACFileReader.Read
    what = "FLACDecoder.CopyTo replay" if wl.fmt_name == "FLACDECODER" else f"FLACFileReader.Read replay ({buf_len} B reads)"
    mss1, passes1, el1 = cpu_baseline(wl.data, wl.fmt_name, buf_len, wl.samples1, max(1.0, budget_s / 4), 1)
    mss, passes, el = cpu_baseline(wl.data, wl.fmt_name, buf_len, wl.samples1, budget_s, nthr)
    return {"value": round(mss, 3), "unit": "MSamples/s", "cores": nthr, "kind": "port",
            "cores_note": f"threads = the host cores available to this process: affinity mask {affinity_cores()}, "
                          f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')} (the box's CPU share per GPU)",
            "sample": f"{passes} x one {wl.cfg} stream ({wl.nf1} frames, {wl.samples1} samples) through the oracle's "
                      f"{what} on {nthr} threads, {el:.1f} s",
            "single_thread": {"value": round(mss1, 3), "cores": 1, "passes": passes1, "seconds": round(el1, 2)},
            "cpu": cpu_model()}


# --------------------------------------------------------------------------- side measurements
def pcie_inclusive(wl, nb=8, reps=3):
    """Host-resident caller: pinned host compressed bytes -> H2D -> parse+decode -> D2H PCM.
    Reported beside `value`, never as it."""
    torch, dev, lf, dec = wl.torch, wl.dev, wl.libflac, wl.dec
    nb = min(nb, wl.B)
    copy_len = wl.copy_len
    h_in = torch.zeros(copy_len * nb + 64, dtype=torch.uint8).pin_memory()
    h_in[:copy_len * nb].copy_(wl.d_bytes[:copy_len * nb].cpu())
    h_out = torch.empty(wl.pcm1 * nb, dtype=torch.uint8).pin_memory()
    d_in = torch.empty_like(h_in, device=dev)
    d_out = torch.empty(wl.pcm1 * nb, dtype=torch.uint8, device=dev)
    nf = wl.nf1 * nb
    d_info = torch.zeros(nf * lf.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def once():
        d_in.copy_(h_in, non_blocking=True)
        dec.decode_frames(d_in, copy_len * nb, wl.d_offs[:nf], nf, wl.sp, wl.fmt, d_out, d_info,
                          d_out_sample=wl.d_os[:nf], stream=stream)
        h_out.copy_(d_out, non_blocking=True)

    once()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ok = h_out[:wl.pcm1].numpy().tobytes() == wl.ref
    return {"value": round(wl.samples1 * nb * reps / el / 1e6, 2), "unit": "MSamples/s",
            "batches": nb * reps, "bitexact": bool(ok),
            "note": "pinned host bytes -> H2D -> k_parse+decode -> D2H PCM, serialized on one stream"}


def index_leg(wl, reps=5):
    """bnflac_index_stream over one whole stream in HBM: sync scan, candidate
    parse, CRC-16 chain.  Wall time per call (it syncs once for the candidate count)."""
    torch, dev, dec = wl.torch, wl.dev, wl.dec
    n = len(wl.data)
    d = torch.zeros((n + 15) // 16 * 16 + 16, dtype=torch.uint8, device=dev)
    d[:n] = torch.from_numpy(np.frombuffer(wl.data, dtype=np.uint8).copy()).to(dev)
    cap = len(wl.offs) + 16
    o, _, _, nf = dec.index_stream(d, n, int(wl.offs[0]), wl.sp, cap)
    match = nf == len(wl.offs) and bool(np.array_equal(o[:nf].cpu().numpy(), wl.offs))
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        dec.index_stream(d, n, int(wl.offs[0]), wl.sp, cap)
    ms = (time.perf_counter() - t0) / reps * 1e3
    return {"ms": round(ms, 4), "GB_per_s": round(n / (ms * 1e-3) / 1e9, 2), "frames": nf, "stream_bytes": n,
            "matches_generator_offsets": match,
            "note": "one stream: sync scan + k_parse of every candidate + CRC-16 chain (one host sync)"}


def reader_leg(wl, reps=3, chunk=16384):
    """bnflac_reader over one whole stream held in host memory: open (H2D, frame
    index, decode-ahead) + Read() in OpenAL-sized 16 KiB pieces until the end.  Reported beside
    `value`, not part of it."""
    lf = wl.libflac
    best, ok = None, True
    for _ in range(reps):
        t0 = time.perf_counter()
        r = lf.Reader(wl.data, wl.fmt)
        got = r.read_all(chunk)
        r.close()
        el = time.perf_counter() - t0
        ok = ok and got == wl.ref
        best = el if best is None else min(best, el)
    out = {"value": round(wl.samples1 / best / 1e6, 2), "unit": "MSamples/s", "ms": round(best * 1e3, 2),
           "bitexact": bool(ok), "read_bytes": chunk,
           "note": "Python ctypes loop: host bytes -> bnflac_reader_open (H2D, index, one decode launch) -> "
                   "Read() x 16 KiB until EOS"}
    exe = os.path.join(ROOT, "tools", "reader_bench")
    if os.path.exists(exe):  # the same pass driven from C (tools/reader_bench.c, built by build())
        import subprocess
        import tempfile
        with tempfile.NamedTemporaryFile(suffix=".flac", delete=False) as tf:
            tf.write(wl.data)
        try:
            r = subprocess.run([exe, tf.name, "10", str(chunk), str(wl.fmt)], capture_output=True, text=True,
                               timeout=120)
            if r.returncode == 0:
                c = json.loads(r.stdout.strip().splitlines()[-1])
                out["from_c"] = {"value": c["MSamples_per_s"], "ms": c["total_ms"], "open_ms": c["open_ms"],
                                 "read_ms": c["read_ms"], "close_ms": c["close_ms"],
                                 "note": "tools/reader_bench: best of 10 open + read x 16 KiB + close"}
        finally:
            os.unlink(tf.name)
    return out


def leg(cfg, args, torch, dev, libflac, synth, dec, stream):
    """One side config on this GPU: value, decode-launch roofline, step roofline, cpu_baseline.
    C5: c5_job at one rank (the config's 8 distinct files in one launch pair), its cpu_baseline
    on a sample of one of them."""
    c = CONFIGS[cfg]
    if cfg == "C5":
        r = c5_job(args, torch, None, dev, libflac, synth, dec, 1, 0, files=c["batches"], steps=args.leg_steps,
                   warmup=1)
        out = c5_summary(r, args, 1, steps=args.leg_steps)
        for k in ("with_gather", "with_gather_overlapped", "with_gather_in_step", "ranks"):
            out.pop(k, None)
        # one file: the per-rank work of C5 at N = 8 (one file per GPU), and what it implies
        r1 = c5_job(args, torch, None, dev, libflac, synth, dec, 1, 0, files=1, steps=args.leg_steps, warmup=1)
        one_ms = r1["t_dec"] / args.leg_steps * 1e3
        out["one_file"] = {"ms_per_step": round(one_ms, 4), "parse_ms": round(r1["t_parse"], 4),
                           "decode_ms": round(r1["t_decode"], 4), "bitexact": r1["ok"],
                           "projected_8gpu_speedup": round(out["ms_per_step"] / one_ms, 3),
                           "note": "PROJECTION, not a measurement of 8 GPUs: one file's step on this GPU is each "
                                   "rank's work at N = 8; speedup = the 8-file step here / that (gather excluded)"}
        out["steps"] = args.leg_steps
        out["config"] = {"workload": c["desc"], "files": r["files"], "frames_per_step": r["frames_rank"]}
        if not args.no_cpu_baseline:
            wl = Workload(cfg, 1, 0, torch, dev, libflac, synth, dec)
            out["cpu_baseline"] = cpu_leg(wl, args.leg_cpu_seconds, args.cpu_threads)
            del wl
        torch.cuda.empty_cache()
        return out
    wl = Workload(cfg, c["batches"], 0, torch, dev, libflac, synth, dec)
    el, tp, td = timed(wl, args.leg_steps, 1, stream, 1, None, dev)
    ok = wl.check()
    step_ms = el / args.leg_steps * 1e3
    out = {"value": round(wl.samples * args.leg_steps / el / 1e6, 2), "unit": "MSamples/s",
           "ms_per_step": round(step_ms, 4), "steps": args.leg_steps, "bitexact": ok,
           "config": {"workload": c["desc"], "frames_per_batch": wl.nf1, "batches_per_step": wl.B,
                      "compressed_bytes_per_batch": wl.fb_in, "pcm_bytes_per_batch": wl.pcm1},
           "roofline": roofline(wl.alg_bytes, td, tp, step_ms, measured_traffic(cfg, wl.B, wl.nf1))}
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_leg(wl, args.leg_cpu_seconds, args.cpu_threads)
    del wl
    torch.cuda.empty_cache()
    return out


# --------------------------------------------------------------------------- C5: files over ranks
def c5_job(args, torch, dist, dev, libflac, synth, dec, world, rank, files=None, steps=None, warmup=None):
    """C5 as BASELINE.json states it: F files of 192 kHz/24-bit 8-channel LPC-32 audio sharded
    over the ranks (shard.partition by samples), each rank indexing its files on the GPU
    (bnflac_index_stream, untimed setup) and decoding them (timed: k_parse + decode launch over
    all its files at once), then the FLACFileReader PCM gathered to rank 0 (shard.gather_bytes:
    concurrent RCCL receives over xGMI)."""
    from birdnest.audio_amd import shard
    F = files or args.batches or CONFIGS["C5"]["batches"]
    steps = steps or args.steps
    warmup = args.warmup if warmup is None else warmup
    p0 = synth.config("C5")
    ranges = shard.partition([p0.nframes * p0.blocksize] * F, world)  # equal files: F/world each
    # The rank-local setup (generate, index, warm up) fails, if at all, on one rank alone: every
    # rank then learns it at one all_reduce that all of them reach, and all raise together, so
    # no rank is left waiting in a later collective (main() reports the error in the C5 leg).
    err = None
    try:
        lo, hi = ranges[rank]
        mine = list(range(lo, hi))
        streams = [synth.encode(synth.config("C5", seed=5 + 1000 * i)) for i in mine]
        sp = libflac.StreamParams.from_synth(p0, streams[0].nsamples if streams else 0)
        fmt = libflac.OUT_FILEREADER
        stride = libflac.out_stride(fmt, sp)
        lens = [(len(s.data) + 255) // 256 * 256 for s in streams]
        base = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64) if streams else np.zeros(1, np.int64)
        d_bytes = torch.zeros(int(base[-1]) + 64, dtype=torch.uint8, device=dev)
        offs, osmp, nsmp = [], [], 0
        for i, s in enumerate(streams):
            n = len(s.data)
            d_bytes[int(base[i]):int(base[i]) + n] = torch.from_numpy(s.data.copy()).to(dev)
            o, os_, _, nf = dec.index_stream(d_bytes[int(base[i]):], n, int(s.frame_offsets[0]), sp, len(s.frame_offsets) + 8)
            assert nf == len(s.frame_offsets), "GPU frame index disagrees with the generator"
            offs.append(o[:nf].cpu().numpy() + int(base[i]))
            osmp.append(os_[:nf].cpu().numpy() + nsmp)
            nsmp += s.nsamples
        nframes = int(sum(len(o) for o in offs))
        d_offs = torch.from_numpy(np.concatenate(offs) if offs else np.zeros(0, np.int64)).to(dev)
        d_os = torch.from_numpy(np.concatenate(osmp) if osmp else np.zeros(0, np.int64)).to(dev)
        d_out = torch.empty(max(nsmp * stride, 1), dtype=torch.uint8, device=dev)
        d_out2 = torch.empty_like(d_out)  # the overlapped flow's second output buffer
        d_info = torch.zeros(max(nframes, 1) * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
        stream = torch.cuda.current_stream(dev)
        nb = int(base[-1])

        def decode(out=d_out, e=None):
            if nframes:
                dec.parse_frames(d_bytes, nb, d_offs, nframes, sp, d_info, d_out_sample=d_os, stream=stream)
                if e is not None:
                    e[1].record(stream)
                dec.decode_parsed(d_bytes, nb, nframes, sp, fmt, out, d_info, stream=stream)

        for _ in range(warmup):
            decode()
        torch.cuda.synchronize(dev)
    except Exception as e:  # noqa: BLE001 -- re-raised below on every rank
        err = f"rank {rank}: {type(e).__name__}: {e}"
    if world > 1:
        flag = torch.tensor([0 if err else 1], device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if not int(flag.item()):
            raise RuntimeError(err or "C5 setup failed on another rank")
    elif err:
        raise RuntimeError(err)
    if world > 1:
        dist.barrier()
    ev = []
    t0 = time.perf_counter()
    for _ in range(steps):
        e = tuple(torch.cuda.Event(enable_timing=True) for _ in range(3))
        e[0].record(stream)
        e[1].record(stream)  # re-recorded between the two launches when there are frames
        decode(e=e)
        e[2].record(stream)
        ev.append(e)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t_dec = time.perf_counter() - t0
    t_launch = sum(a.elapsed_time(c) for a, _, c in ev) / len(ev)
    t_parse = sum(a.elapsed_time(b) for a, b, _ in ev) / len(ev)
    t_decode = sum(b.elapsed_time(c) for _, b, c in ev) / len(ev)
    # decode + gather: the same steps, each followed by the gather of every rank's PCM to rank 0
    gathered = None
    t0 = time.perf_counter()
    for _ in range(steps):
        decode()
        if world > 1:
            gathered = shard.gather_bytes(d_out[:nsmp * stride])
        else:
            gathered = d_out[:nsmp * stride]
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t_all = time.perf_counter() - t0
    # decode + gather, overlapped across steps: step s decodes into one of two output buffers
    # and posts its gather (shard.gather_post: RCCL point-to-point ops ordered after that
    # decode); step s + 1's decode into the other buffer runs while it is in flight, and a
    # buffer is decoded into again only after its previous gather finished (work.wait)
    t_ovl = t_all
    gathered_ovl = None
    if world > 1:
        nbytes_out = nsmp * stride
        sizes = shard.gather_sizes(d_out[:nbytes_out])
        bufs, pend, parts = [d_out, d_out2], [[], []], [None, None]
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for st in range(steps):
            b = st % 2
            for wk in pend[b]:
                wk.wait()
            decode(bufs[b])
            pend[b], parts[b] = shard.gather_post(bufs[b][:nbytes_out], sizes, parts=parts[b])
        for b in (0, 1):
            for wk in pend[b]:
                wk.wait()
        torch.cuda.synchronize(dev)
        dist.barrier()
        t_ovl = time.perf_counter() - t0
        last = (steps - 1) % 2
        if rank == 0 and parts[last] is not None:
            gathered_ovl = torch.cat(parts[last])
    # decode + gather overlapped inside one step: the rank's files decoded one
    # group (file) at a time, each group's PCM posted to rank 0 (shard.GroupGather) as soon as
    # its decode is enqueued, so group g's transfer runs beside group g + 1's decode
    t_grp, gathered_grp = t_all, None
    if world > 1:
        # groups: the rank's files, or (--c5-split K) K frame ranges of each file; a group's
        # bytes run from its first frame's output sample to the next group's
        franges, _ = shard.frame_groups([len(o) for o in offs], getattr(args, "c5_split", 1))
        fstart = np.concatenate(osmp + [np.array([nsmp], np.int64)]) if osmp else np.zeros(1, np.int64)
        gb = [(int(fstart[a]) * stride, int(fstart[b]) * stride) for a, b in franges]
        gsz = shard.gather_group_sizes([b - a for a, b in gb], device=dev)

        def grouped():
            gg = shard.GroupGather(gsz, d_out)
            for g, (f0, f1) in enumerate(franges):
                if f1 > f0:
                    di = d_info[f0 * libflac.FRAME_INFO_BYTES:f1 * libflac.FRAME_INFO_BYTES]
                    dec.parse_frames(d_bytes, nb, d_offs[f0:f1], f1 - f0, sp, di, d_out_sample=d_os[f0:f1], stream=stream)
                    dec.decode_parsed(d_bytes, nb, f1 - f0, sp, fmt, d_out, di, stream=stream)
                gg.post(g, d_out[gb[g][0]:gb[g][1]])
            return gg.wait()

        grouped()
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            gathered_grp = grouped()
        torch.cuda.synchronize(dev)
        dist.barrier()
        t_grp = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([t_dec, t_all, t_ovl, t_grp], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_dec, t_all, t_ovl, t_grp = float(t[0].item()), float(t[1].item()), float(t[2].item()), float(t[3].item())
    ok = True
    if rank == 0:
        local = dict(zip(mine, streams))
        ref = b"".join(pack_reference((local[i] if i in local else synth.encode(synth.config("C5", seed=5 + 1000 * i))).pcm,
                                      "FILEREADER", 24) for i in range(F))
        ok = gathered is not None and gathered.cpu().numpy().tobytes() == ref
        if world > 1:
            ok = ok and gathered_ovl is not None and gathered_ovl.cpu().numpy().tobytes() == ref
            ok = ok and gathered_grp is not None and gathered_grp.cpu().numpy().tobytes() == ref
    if world > 1:
        o = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(o, op=dist.ReduceOp.MIN)
        ok = bool(o.item())
    samples = sum(s.nsamples for s in streams) * p0.channels
    tot = torch.tensor([samples], dtype=torch.int64, device=dev)
    if world > 1:
        dist.all_reduce(tot)
    samples = int(tot.item())
    comp = sum(len(s.data) - int(s.frame_offsets[0]) for s in streams)
    alg = comp + nsmp * stride
    return {"samples": samples, "t_dec": t_dec, "t_all": t_all, "t_ovl": t_ovl, "t_grp": t_grp, "t_launch": t_launch, "ok": ok,
            "t_parse": t_parse, "t_decode": t_decode,
            "files": F, "alg_bytes_rank": alg, "frames_rank": nframes}


def c5_summary(r, args, world, steps=None):
    """value / timing / roofline fields of a c5_job result (the --config C5 line, the C5 leg at
    N = 1, or the C5 flow leg of a multi-GPU C2 run)."""
    steps = steps or args.steps
    step_ms = r["t_dec"] / steps * 1e3
    out = {"value": round(r["samples"] * steps / r["t_dec"] / 1e6, 2), "unit": "MSamples/s",
           "ms_per_step": round(step_ms, 4), "bitexact": r["ok"], "files": r["files"], "ranks": world,
           "roofline": roofline(r["alg_bytes_rank"], r["t_decode"], r["t_parse"], step_ms,
                                measured_traffic("C5", r["files"], CONFIGS["C5"]["frames"]) if world == 1 else None),
           "with_gather": {"value": round(r["samples"] * steps / r["t_all"] / 1e6, 2), "unit": "MSamples/s",
                           "ms_per_step": round(r["t_all"] / steps * 1e3, 4),
                           "note": "each step: decode, then shard.gather_bytes of every rank's PCM to rank 0"},
           "with_gather_overlapped": {"value": round(r["samples"] * steps / r["t_ovl"] / 1e6, 2),
                                      "unit": "MSamples/s", "ms_per_step": round(r["t_ovl"] / steps * 1e3, 4),
                                      "note": "step s's gather (shard.gather_post, RCCL send/recv) in flight while "
                                              "step s + 1 decodes into a second buffer; N = 1: no gather"},
           "with_gather_in_step": {"value": round(r["samples"] * steps / r["t_grp"] / 1e6, 2),
                                   "unit": "MSamples/s", "ms_per_step": round(r["t_grp"] / steps * 1e3, 4),
                                   "note": "one step: the rank's files decoded one at a time, each file's PCM "
                                           "posted to rank 0 (shard.GroupGather) as soon as its decode is "
                                           "enqueued; N = 1: no gather"}}
    out["roofline"]["kernel"] = "decode launch over the rank's files (k_parse beside it: k_parse_avg_ms)"
    out["roofline"]["parse_plus_decode_ms"] = round(r["t_launch"], 4)
    return out


# --------------------------------------------------------------------------- main
def main():
    args = parse_args()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    if args.rank_selftest:
        rank_selftest(args)
        return
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    assert args.gpus is None or args.gpus == world, "rank count differs from --gpus"
    args.gpus = world
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import datetime
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # a stuck collective (barrier, timing reduction, the C5 gather) must end the run with a
        # non-zero exit instead of hanging it: the watchdog aborts after the timeout
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank),
                                timeout=datetime.timedelta(seconds=args.nccl_timeout))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    from birdnest.audio_amd import libflac, synth
    dec = libflac.BatchDecoder(local_rank)
    stream = torch.cuda.current_stream(dev)
    cfg = args.config
    c = CONFIGS[cfg]

    if cfg == "C5" and not args.c5_batch:
        r = c5_job(args, torch, dist, dev, libflac, synth, dec, world, rank)
        line = {"metric": METRIC}
        line.update(c5_summary(r, args, world))
        line.update({"n_gpus": world, "steps": args.steps, "warmup": args.warmup, "higher_is_better": True,
                     "scaling": "strong", "vs_baseline": None, "dtype": "int32",
                     "data": "synthetic: deterministic generator (seeds 5 + 1000 i), BASELINE C5 file shape",
                     "config": {"workload": c["desc"] + f"; {r['files']} files sharded over {world} rank(s), "
                                                         "decode-only timing (gather reported beside it)",
                                "files": r["files"],
                                "parallelism": f"files sharded per rank x{world} + RCCL gather to rank 0"}})
        if rank == 0:
            js = json.dumps(line)
            print(js, flush=True)
            if args.out:
                open(args.out, "w").write(js + "\n")
        if world > 1:
            dist.destroy_process_group()
        return

    # The job's corpus: world x B batches, cut into contiguous ranges by shard.partition (equal
    # batches: B per rank, weak scaling); rank r's batches hold its own stream (seed + 7919 r,
    # rank 0 the config's stream), so no two ranks decode the same bytes.
    from birdnest.audio_amd import shard
    B = args.batches or c["batches"]
    b0, b1 = shard.partition([1] * (world * B), world)[rank]
    seed0 = 2 if cfg == "C2" else synth.config(cfg).seed
    wl = Workload(cfg, b1 - b0, args.frames, torch, dev, libflac, synth, dec, seed=seed0 + 7919 * rank)
    elapsed, t_parse, t_decode = timed(wl, args.steps, args.warmup, stream, world, dist, dev)
    ok = wl.check()
    if world > 1:
        o = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(o, op=dist.ReduceOp.MIN)
        ok = bool(o.item())
    step_ms = elapsed / args.steps * 1e3
    samples = wl.samples
    if world > 1:  # every rank's own count (its stream's samples)
        t = torch.tensor([samples], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        samples = int(t.item())
    value = samples * args.steps / elapsed / 1e6
    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "MSamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": f"synthetic: deterministic generator, BASELINE {cfg} frame shape",
        "config": {"workload": c["desc"], "frames_per_batch": wl.nf1, "batches_per_step": B,
                   "compressed_bytes_per_batch": wl.fb_in, "pcm_bytes_per_batch": wl.pcm1,
                   "parallelism": f"corpus of {world} x {B} batches partitioned per rank (shard.partition) x{world}"},
        "per_gpu_value": round(value / world, 2),
        "bitexact": ok,
        "roofline": roofline(wl.alg_bytes, t_decode, t_parse, step_ms, measured_traffic(cfg, B, wl.nf1)),
        "kernels_sha": kernels_sha(),
    }
    if args.stats and rank == 0:
        import ctypes
        buf = (ctypes.c_uint64 * 16)()
        dec.L.bnflac_debug_stats(buf, 1)
        dec.L.bnflac_debug_set_ablate(0x100)
        wl.run(1, stream)
        torch.cuda.synchronize(dev)
        dec.L.bnflac_debug_stats(buf, 1)
        dec.L.bnflac_debug_set_ablate(0)
        names = ["fused_chunks", "generic_chunks", "dma_land_waits", "slow_rice", "refills", "waves"]
        line["stats"] = {n: int(buf[i]) for i, n in enumerate(names)}
        w = max(1, int(buf[5]))
        line["stats"]["cycles_per_wave"] = {n: int(buf[8 + i]) // w for i, n in
                                            enumerate(["setup", "decode", "refill", "pack", "tail"])}
        # k_decode_sys (BNFLAC_DECODE_SYS=1): s_memtime per producer wave / per restore wave
        line["stats"]["sys_cycles"] = {n: int(buf[8 + i]) // w for i, n in
                                       enumerate(["prod_refill", "prod_rice", "prod_barrier", "rest_steps",
                                                  "rest_pack", "rest_barrier", "refill_wait", "dma_in_flight"])}
    if args.ablate and rank == 0:
        abl = []
        for m in [int(x, 0) for x in args.ablate.split(",")]:
            dec.L.bnflac_debug_set_ablate(m)
            wl.run(1, stream)
            pe, de = [], []
            wl.run(args.steps, stream, pe, de)
            torch.cuda.synchronize(dev)
            abl.append({"ablate": m, "k_parse_ms": round(sum(a.elapsed_time(b) for a, b in pe) / len(pe), 4),
                        "k_decode_ms": round(sum(a.elapsed_time(b) for a, b in de) / len(de), 4)})
        dec.L.bnflac_debug_set_ablate(0)
        line["ablation"] = abl
    if rank == 0 and not args.no_index:
        line["indexer"] = index_leg(wl)
    if rank == 0 and not args.no_reader:
        line["reader"] = reader_leg(wl)
    if rank == 0 and not args.no_pcie:
        line["pcie_inclusive"] = pcie_inclusive(wl)
    if rank == 0 and not args.no_cpu_baseline:
        sys.stdout.flush()
        line["cpu_baseline"] = cpu_leg(wl, args.cpu_seconds, args.cpu_threads)
    legs = [x for x in args.legs.split(",") if x and x != cfg] if world == 1 else []
    if legs:
        del wl
        torch.cuda.empty_cache()
        line["legs"] = {x: leg(x, args, torch, dev, libflac, synth, dec, stream) for x in legs}
    elif world > 1 and not args.no_c5_flow:
        # BASELINE config 5 at N GPUs: the files sharded over the ranks, each rank indexing and
        # decoding its own, then the gather of every rank's PCM to rank 0 over RCCL
        del wl
        torch.cuda.empty_cache()
        try:  # the headline above is measured: an error in the side flow must not lose its line
            r = c5_job(args, torch, dist, dev, libflac, synth, dec, world, rank)
            line["legs"] = {"C5_flow": c5_summary(r, args, world)}
            line["legs"]["C5_flow"]["config"] = {"workload": CONFIGS["C5"]["desc"], "files": r["files"],
                                                 "parallelism": f"files sharded per rank x{world} + RCCL gather to rank 0"}
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line, never swallowed
            line["legs"] = {"C5_flow": {"error": f"{type(e).__name__}: {e}"[:500]}}
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
