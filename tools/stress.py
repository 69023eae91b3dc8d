"""Randomised stress run (not a unit test): N synthetic streams with every generator knob
drawn at random, decoded through the batch API in two layouts and checked bit-exact
against the CPU oracle's decode (the parity reference; the generator's source PCM is used
when the two agree, and the few streams where the generator's own PCM is off -- 8-bit
constant frames out of range -- are reported separately).  usage: python tools/stress.py [N] [seed0]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from birdnest.audio_amd import libflac, synth

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle  # noqa: E402  (test infrastructure: the reference for this check)


def draw(rng):
    ch = int(rng.choice([1, 2, 2, 2, 3, 6, 8]))
    bps = int(rng.choice([8, 12, 16, 16, 16, 20, 24]))
    var = int(rng.integers(0, 4) == 0)
    bs = int(rng.choice([192, 576, 1152, 2048, 4096, 4608, 8192]))
    mode = int(rng.choice([synth.SUB_LPC, synth.SUB_LPC, synth.SUB_FIXED, synth.SUB_MIXED, synth.SUB_VERBATIM]))
    kw = dict(channels=ch, bps=bps, blocksize=bs, nframes=int(rng.integers(8, 90)), last_blocksize=int(rng.integers(16, bs)),
              subframe_mode=mode, order=int(rng.integers(1, 33 if mode == synth.SUB_LPC else 9)),
              partition_order=int(rng.choice([-1, 0, 1, 3, 5])), stereo_mode=int(rng.integers(0, 5)) if ch == 2 else 0,
              rice2=int(rng.integers(0, 2)), escape_permille=int(rng.choice([0, 0, 30])),
              wasted_bits_max=int(rng.choice([0, 0, 2, 5])), level=float(rng.uniform(0.02, 0.95)),
              noise=float(rng.choice([0.0003, 0.004, 0.03, 0.3])), seed=int(rng.integers(1, 1 << 30)),
              prec_clamp=int(rng.integers(0, 2)), variable_blocksize=var, impulse_permille=int(rng.choice([0, 0, 0, 2])),
              sample_rate=int(rng.choice([8000, 44100, 48000, 96000, 192000])))
    if mode == synth.SUB_FIXED:
        kw["order"] = int(rng.integers(0, 5))
    if var:
        kw["bs_min"], kw["bs_max"] = 192, int(rng.choice([4096, 16384]))
    return kw


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    rng = np.random.default_rng(seed0)
    dec = libflac.BatchDecoder(0)
    dev = torch.device("cuda:0")
    bad = 0
    t0 = time.time()
    for i in range(n):
        kw = draw(rng)
        try:
            s = synth.encode(synth.config("C2", **kw))
        except Exception as e:  # the generator refuses a few combinations
            print(i, "generator refused", kw, e)
            continue
        data = s.data.tobytes()
        if "--corrupt" in sys.argv:  # damaged stream: only the stream API's error handling is compared
            buf = bytearray(data)
            first = int(s.frame_offsets[0])
            for _ in range(int(rng.integers(1, 6))):
                pos = int(rng.integers(first, len(buf)))
                buf[pos] ^= int(rng.integers(1, 256))
            if rng.integers(0, 4) == 0:
                buf = buf[: int(rng.integers(first, len(buf)))]  # truncated too
            data = bytes(buf)
            from birdnest.audio_amd import harness
            ok = True
            for drv in (0, 1):
                ev, opcm = oracle.run(data, driver=drv)
                hev, hpcm = harness.run(data, driver=drv)
                if hev != harness.oracle_events_as_tuples(ev) or not np.array_equal(hpcm, opcm):
                    ok = False
                    print(i, "corrupt stream: stream API differs from the oracle, driver", drv, flush=True)
                    break
            if not ok:
                bad += 1
                print(i, "MISMATCH", kw, flush=True)
            if i % 20 == 0:
                print(i, "ok so far, bad", bad, f"{time.time() - t0:.0f}s", flush=True)
            continue
        ev, opcm = oracle.run(data)
        ref = oracle.interleave(ev, opcm)
        if ref.shape != s.pcm.shape or not np.array_equal(ref, s.pcm):
            print(i, "generator PCM differs from the oracle (reference = oracle)", flush=True)
        if ref.shape != s.pcm.shape:
            continue
        sp = libflac.StreamParams.from_synth(s.params, s.nsamples)
        nb = len(data)
        d_bytes = torch.zeros((nb + 15) // 16 * 16 + 16, dtype=torch.uint8, device=dev)
        d_bytes[:nb] = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(dev)
        offs = torch.from_numpy(s.frame_offsets.astype(np.int64)).to(dev)
        nf = len(s.frame_offsets)
        ok = True
        for fmt in (libflac.OUT_INTERLEAVED32, libflac.OUT_PLANAR32):
            stride = libflac.out_stride(fmt, sp)
            d_out = torch.zeros(int(s.nsamples) * stride + 64, dtype=torch.uint8, device=dev)
            d_info = torch.zeros(nf * 128, dtype=torch.uint8, device=dev)
            dec.decode_frames(d_bytes, nb, offs, nf, sp, fmt, d_out, d_info)
            torch.cuda.synchronize()
            info = libflac.info_array(d_info.cpu().numpy())
            if not ((info["status"] == 0).all() and (info["crc_ok"] == 1).all()):
                badf = np.nonzero((info["status"] != 0) | (info["crc_ok"] != 1))[0]
                print(i, "fmt", fmt, "frame status/crc", badf[:5].tolist(), info["status"][badf[:5]].tolist(),
                      info["err"][badf[:5]].tolist(), info["flags"][badf[:5]].tolist(), flush=True)
                ok = False
                break
            out = d_out.cpu().numpy()[: int(s.nsamples) * stride].view("<i4")
            if fmt == libflac.OUT_INTERLEAVED32:
                ok = np.array_equal(out.reshape(-1, s.pcm.shape[1]), ref)
            else:
                o = 0
                for fr in range(nf):
                    b = int(info["blocksize"][fr])
                    st = int(info["out_sample"][fr])
                    if not np.array_equal(out[o: o + b * s.pcm.shape[1]].reshape(s.pcm.shape[1], b).T, ref[st: st + b]):
                        ok = False
                        break
                    o += b * s.pcm.shape[1]
            if not ok:
                print(i, "fmt", fmt, "PCM differs", flush=True)
                break
        if ok and "--index" in sys.argv:  # GPU frame chain == the generator's frame offsets
            offs_i, _, _, nfi = dec.index_stream(d_bytes, nb, int(s.frame_offsets[0]), sp, nf + 16)
            if nfi != nf or not np.array_equal(offs_i[:nf].cpu().numpy(), s.frame_offsets.astype(np.int64)):
                print(i, "index differs", nfi, nf, flush=True)
                ok = False
        if ok and "--layouts" in sys.argv and kw["bps"] == 16:  # FLACDecoder bytes == the C# replay
            orc, oref, omsg, _ = oracle.flacdecoder_copyto(data)
            if orc == 0:
                stride = libflac.out_stride(libflac.OUT_FLACDECODER, sp)
                d_out = torch.zeros(int(s.nsamples) * stride + 64, dtype=torch.uint8, device=dev)
                d_info = torch.zeros(nf * 128, dtype=torch.uint8, device=dev)
                dec.decode_frames(d_bytes, nb, offs, nf, sp, libflac.OUT_FLACDECODER, d_out, d_info)
                torch.cuda.synchronize()
                if d_out.cpu().numpy()[: int(s.nsamples) * stride].tobytes() != oref:
                    print(i, "FLACDecoder layout differs from the C# replay", flush=True)
                    ok = False
        if ok and "--reader" in sys.argv and kw["bps"] == 16:  # streaming reader == the C# CopyTo replay
            orc, oref, omsg, _ = oracle.flacdecoder_copyto(data)
            if orc == 0:
                r = libflac.Reader(data, libflac.OUT_FLACDECODER, window_frames=int(rng.integers(1, 64)))
                got = r.read_all(int(rng.choice([1000, 16384, 65536])))
                r.close()
                if got != oref:
                    print(i, "reader differs from the C# replay", flush=True)
                    ok = False
        if ok and "--api" in sys.argv:  # libFLAC-compatible stream API events == the oracle's
            from birdnest.audio_amd import harness
            hev, hpcm = harness.run(data, driver=0)
            if hev != harness.oracle_events_as_tuples(ev) or not np.array_equal(hpcm, opcm):
                print(i, "stream API differs from the oracle", flush=True)
                ok = False
        if not ok:
            bad += 1
            print(i, "MISMATCH", kw, flush=True)
        if i % 20 == 0:
            print(i, "ok so far, bad", bad, f"{time.time() - t0:.0f}s", flush=True)
    print("done", n, "streams, bad", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
