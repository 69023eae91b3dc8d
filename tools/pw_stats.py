#!/usr/bin/env python3
"""k_parse_wave vs k_parse on one config's frames (timing + the wave scan's debug counters).

    BNFLAC_PW_STATS=1 python tools/pw_stats.py [C5|C2|C3] [copies]
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
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C5"
    copies = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    p = synth.config(cfg, **({"last_blocksize": 0} if cfg == "C5" else {}))
    s = synth.encode(p)
    data = s.data.tobytes()
    cl = (len(data) + 255) // 256 * 256
    dev = torch.device("cuda:0")
    one = np.zeros(cl, np.uint8)
    one[:len(data)] = np.frombuffer(data, np.uint8)
    d_bytes = torch.from_numpy(np.tile(one, copies)).to(dev)
    offs = np.concatenate([s.frame_offsets.astype(np.int64) + i * cl for i in range(copies)])
    d_offs = torch.from_numpy(offs).to(dev)
    nf = len(offs)
    sp = libflac.StreamParams.from_synth(p, s.nsamples)
    L = libflac.load()
    dec = libflac.BatchDecoder(0)
    res = {}
    for mode in (0, 1, 0, 1):
        L.bnflac_debug_set_parse_wave(mode)
        d_info = torch.zeros(nf * libflac.FRAME_INFO_BYTES, dtype=torch.uint8, device=dev)
        dec.parse_frames(d_bytes, cl * copies, d_offs, nf, sp, d_info)
        torch.cuda.synchronize()
        buf = (ctypes.c_uint64 * 8)()
        L.bnflac_debug_parse_wave_stats(buf, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            dec.parse_frames(d_bytes, cl * copies, d_offs, nf, sp, d_info)
        e1.record()
        torch.cuda.synchronize()
        L.bnflac_debug_parse_wave_stats(buf, 1)
        res[mode] = (e0.elapsed_time(e1) / 5, d_info.cpu().numpy())
        print(f"{cfg} x{copies} ({nf} frames) parse mode {mode}: {res[mode][0]:.3f} ms", flush=True)
        if mode == 1:
            v = [int(x) / 5 for x in buf]
            print("  per launch: passes %.0f, splice rounds %.0f, serial fallbacks %.0f, partitions %.0f, frames %.0f,"
                  " scan wave-cycles %.3g (%.0f per pass: %.0f window waits, %.0f splice)" % (
                      v[0], v[1], v[2], v[3], v[4], v[5], v[5] / max(v[0], 1), v[6] / max(v[0], 1), v[7] / max(v[0], 1)))
    print("records identical:", np.array_equal(res[0][1], res[1][1]))


if __name__ == "__main__":
    main()
