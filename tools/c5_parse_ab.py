#!/usr/bin/env python3
"""C5 parse A/B (VERDICT r4 "next" 3): k_parse_wave over 8 copies of one file against 8 distinct
files (the bench's c5_job seeds), and each distinct file alone, with the wave scan's debug
counters (passes, splice rounds, serial fallbacks).  Also times one file's parse + decode.

    BNFLAC_PW_STATS=1 python tools/c5_parse_ab.py
    BNFLAC_PW_SEG=-1: small partitions through wave passes too (no scalar walk; A/B)
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from birdnest.audio_amd import libflac, synth
    dev = torch.device("cuda:0")
    L = libflac.load()
    dec = libflac.BatchDecoder(0)
    p0 = synth.config("C5")
    streams = {seed: synth.encode(synth.config("C5", seed=seed)) for seed in [5 + 1000 * i for i in range(8)]}

    def build(seeds):
        ss = [streams[s] for s in seeds]
        lens = [(len(s.data) + 255) // 256 * 256 for s in ss]
        base = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        buf = np.zeros(int(base[-1]) + 64, np.uint8)
        offs, osmp, n = [], [], 0
        for i, s in enumerate(ss):
            buf[base[i]:base[i] + len(s.data)] = s.data
            offs.append(s.frame_offsets.astype(np.int64) + base[i])
            osmp.append(np.arange(len(s.frame_offsets), dtype=np.int64) * p0.blocksize + n)
            n += s.nsamples
        return (torch.from_numpy(buf).to(dev), int(base[-1]), torch.from_numpy(np.concatenate(offs)).to(dev),
                torch.from_numpy(np.concatenate(osmp)).to(dev), n)

    sp = libflac.StreamParams.from_synth(p0, streams[5].nsamples)
    fmt = libflac.OUT_FILEREADER
    stride = libflac.out_stride(fmt, sp)

    def run(name, seeds, reps=10):
        d_bytes, nb, d_offs, d_os, nsmp = build(seeds)
        nf = d_offs.numel()
        d_info = torch.zeros(nf * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
        d_out = torch.empty(nsmp * stride, dtype=torch.uint8, device=dev)
        for _ in range(2):
            dec.parse_frames(d_bytes, nb, d_offs, nf, sp, d_info, d_out_sample=d_os)
            dec.decode_parsed(d_bytes, nb, nf, sp, fmt, d_out, d_info)
        torch.cuda.synchronize()
        buf = (ctypes.c_uint64 * 8)()
        L.bnflac_debug_parse_wave_stats(buf, 1)
        ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(reps)]
        for e in ev:
            e[0].record()
            dec.parse_frames(d_bytes, nb, d_offs, nf, sp, d_info, d_out_sample=d_os)
            e[1].record()
            dec.decode_parsed(d_bytes, nb, nf, sp, fmt, d_out, d_info)
            e[2].record()
        torch.cuda.synchronize()
        L.bnflac_debug_parse_wave_stats(buf, 1)
        tp = sorted(e[0].elapsed_time(e[1]) for e in ev)[reps // 2]
        td = sorted(e[1].elapsed_time(e[2]) for e in ev)[reps // 2]
        v = [int(x) / reps for x in buf]
        info = libflac.info_array(d_info.cpu().numpy())
        ok = bool((info["status"] == 0).all() and (info["crc_ok"] == 1).all())
        ref = b"".join(np.ascontiguousarray(streams[s].pcm.astype("<i4")).view(np.uint8).reshape(-1, 4)[:, :3].tobytes()
                       for s in seeds)
        ok = ok and d_out.cpu().numpy().tobytes() == ref
        print(f"{name:28s} frames {nf:5d}  parse {tp:.3f} ms  decode {td:.3f} ms  total {tp + td:.3f} ms  ok={ok}  "
              f"passes {v[0]:.0f} splice {v[1]:.0f} serial {v[2]:.0f} partitions {v[3]:.0f} scan-cyc {v[5]:.3g} "
              f"win-wait {v[6]:.3g} splice-cyc {v[7]:.3g}", flush=True)

    seeds = [5 + 1000 * i for i in range(8)]
    run("8 copies of seed 5", [5] * 8)
    run("8 distinct (c5_job)", seeds)
    for s in seeds:
        run(f"1 file, seed {s}", [s])
    run("4 distinct", seeds[:4])


if __name__ == "__main__":
    main()
