"""CRC-16 hand-off on a bench-sized batch (development check, GPU): for each crc mode, how many
frames got a verdict / a prefix, and the parse and decode times of the batch (HIP events).

    python tools/crc_handoff_check.py [--copies 64] [--cfg C2]
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="C2")
    ap.add_argument("--copies", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="0,1,2")
    a = ap.parse_args()
    import torch
    from birdnest.audio_amd import libflac, synth
    L = libflac.load()
    s = synth.encode(synth.config(a.cfg))
    data = s.data.tobytes()
    clen = (len(data) + 63) // 64 * 64
    offs1 = np.array([int(x) for x in s.frame_offsets], np.int64)
    dev = torch.device("cuda:0")
    n = clen * a.copies
    host = np.zeros(n + 64, np.uint8)
    for b in range(a.copies):
        host[b * clen: b * clen + len(data)] = np.frombuffer(data, np.uint8)
    d_bytes = torch.from_numpy(host).to(dev)
    offs = np.concatenate([offs1 + b * clen for b in range(a.copies)])
    nf = len(offs)
    d_offs = torch.from_numpy(offs).to(dev)
    bs = s.params.blocksize
    os_ = np.concatenate([np.arange(len(offs1), dtype=np.int64) * bs + b * int(s.nsamples) for b in range(a.copies)])
    d_os = torch.from_numpy(os_).to(dev)
    sp = libflac.StreamParams(1, bs, bs, s.params.sample_rate, s.params.channels, s.params.bps,
                              int(s.nsamples) * a.copies)
    fmt = libflac.OUT_FLACDECODER if s.params.bps == 16 else libflac.OUT_INTERLEAVED32
    stride = libflac.out_stride(fmt, sp)
    d_out = torch.empty(int(s.nsamples) * a.copies * stride + 64, dtype=torch.uint8, device=dev)
    d_info = torch.zeros(nf * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
    dec = libflac.BatchDecoder(0)
    ref = None
    for mode in [int(x) for x in a.modes.split(",")]:
        L.bnflac_debug_set_crc_mode(mode)
        tp, td = [], []
        for r in range(a.reps):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record()
            dec.parse_frames(d_bytes, n, d_offs, nf, sp, d_info, d_out_sample=d_os)
            e[1].record()
            if r == a.reps - 1 and mode:
                h = dec.crc_handoff(nf)
            dec.decode_parsed(d_bytes, n, nf, sp, fmt, d_out, d_info)
            e[2].record()
            torch.cuda.synchronize()
            tp.append(e[0].elapsed_time(e[1]))
            td.append(e[1].elapsed_time(e[2]))
        info = libflac.info_array(d_info.cpu().numpy())
        out = d_out.cpu().numpy()
        if ref is None:
            ref = out
        msg = f"mode {mode}: parse {np.median(tp):.3f} ms decode {np.median(td):.3f} ms, ok {int((info['crc_ok'] == 1).sum())}/{nf}, same PCM {np.array_equal(out, ref)}"
        if mode:
            msg += f", spans {int((h[:, 4] != 0).sum())} verdict1 {int((h[:, 5] == 1).sum())} prefixes {int((h[:, 2] != 0).sum())}"
        print(msg, flush=True)
    L.bnflac_debug_set_crc_mode(-1)


if __name__ == "__main__":
    main()
