"""Replay the MISMATCH lines of a tools/stress.py log on the GPU (debug tool, not a test):
each stream is regenerated from its printed generator knobs, decoded through the batch API
(interleaved32) with the fused k_decode path on and off (ablate 0x800), and compared with
the oracle frame by frame; the first differing frame/channel/sample is printed with the
frame's record.  usage: python tools/dbg_kw.py gpurun_out/stress_x.log [more logs]
BNFLAC_LIB_DIR=<dir> loads libbnflac.so from another build (A/B against an older commit)."""
import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from birdnest.audio_amd import _lib  # noqa: E402

if os.environ.get("BNFLAC_LIB_DIR"):
    _lib.LIB_DIR = os.environ["BNFLAC_LIB_DIR"]
from birdnest.audio_amd import libflac, synth  # noqa: E402
import oracle  # noqa: E402  (test infrastructure: the reference)


def cases(paths):
    for p in paths:
        for line in open(p):
            if " MISMATCH " in line:
                yield line.split()[0], ast.literal_eval(line.split(" MISMATCH ", 1)[1])


def run(dec, data, s, nf, ablate):
    dev = torch.device("cuda:0")
    nb = len(data)
    sp = libflac.StreamParams.from_synth(s.params, s.nsamples)
    d_bytes = torch.zeros((nb + 15) // 16 * 16 + 16, dtype=torch.uint8, device=dev)
    d_bytes[:nb] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
    offs = torch.from_numpy(s.frame_offsets.astype(np.int64)).to(dev)
    stride = libflac.out_stride(libflac.OUT_INTERLEAVED32, sp)
    d_out = torch.zeros(int(s.nsamples) * stride + 64, dtype=torch.uint8, device=dev)
    d_info = torch.zeros(nf * 128, dtype=torch.uint8, device=dev)
    libflac.load().bnflac_debug_set_ablate(ablate)
    dec.decode_frames(d_bytes, nb, offs, nf, sp, libflac.OUT_INTERLEAVED32, d_out, d_info)
    torch.cuda.synchronize()
    libflac.load().bnflac_debug_set_ablate(0)
    info = libflac.info_array(d_info.cpu().numpy())
    return d_out.cpu().numpy()[: int(s.nsamples) * stride].view("<i4").reshape(-1, s.pcm.shape[1]), info


def sub_heads(data, rec):
    """(type, order, wasted, rice2, porder) of every subframe of a frame record"""
    bits = np.unpackbits(np.frombuffer(data, np.uint8))
    base = int(rec["frame_off"]) * 8
    out = []
    for c in range(int(rec["channels"])):
        p = base + int(rec["sub_start"][c])

        def rd(n):
            nonlocal p
            v = 0
            for _ in range(n):
                v = (v << 1) | int(bits[p])
                p += 1
            return v
        rd(1)
        t = rd(6)
        wasted = 0
        if rd(1):
            wasted = 1
            while not rd(1):
                wasted += 1
        bps = int(rec["bps"]) - wasted
        a = int(rec["assignment"])
        if (a == 1 and c == 1) or (a == 2 and c == 0) or (a == 3 and c == 1):
            bps += 1
        if t == 0:
            out.append(("CONST", 0, wasted))
            continue
        if t == 1:
            out.append(("VERB", 0, wasted))
            continue
        if t & 0x20:
            order = (t & 31) + 1
            rd(order * bps)
            prec = rd(4) + 1
            shift = rd(5)
            rd(order * prec)
            kind = f"LPC p{prec} s{shift}"
        else:
            order = t & 7
            rd(order * bps)
            kind = "FIXED"
        method = rd(2)
        porder = rd(4)
        out.append((kind, order, wasted, method, porder))
    return out


def main():
    dec = libflac.BatchDecoder(0)
    for idx, kw in cases(sys.argv[1:]):
        s = synth.encode(synth.config("C2", **kw))
        data = s.data.tobytes()
        ev, opcm = oracle.run(data)
        ref = oracle.interleave(ev, opcm)
        nf = len(s.frame_offsets)
        print(f"case {idx}: {nf} frames, {ref.shape}, kw {kw}")
        for ab in (0, 0x800):
            out, info = run(dec, data, s, nf, ab)
            bad = [f for f in range(nf) if info["status"][f] != 0 or info["crc_ok"][f] != 1]
            for f in range(nf):
                st, b = int(info["out_sample"][f]), int(info["blocksize"][f])
                if st + b <= ref.shape[0] and not np.array_equal(out[st: st + b], ref[st: st + b]):
                    d = np.nonzero(out[st: st + b] != ref[st: st + b])
                    bad.append(f)
                    print(f"  ablate {ab:#x}: frame {f} first diff sample {d[0][0]} ch {d[1][0]} "
                          f"got {out[st + d[0][0], d[1][0]]} want {ref[st + d[0][0], d[1][0]]} ndiff {len(d[0])}")
                    break
            bad = sorted(set(bad))
            print(f"  ablate {ab:#x}: bad frames {bad[:8]}")
            for f in bad[:2]:
                print("   record", {k: info[k][f].tolist() for k in info.dtype.names})
                print("   subframes", sub_heads(data, info[f]))


if __name__ == "__main__":
    main()
