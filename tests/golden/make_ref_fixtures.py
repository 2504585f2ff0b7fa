"""Generate the f1/f2 fixtures from the REFERENCE's own logger.

Run from the repo root, in the container that holds /root/reference:
    python tests/golden/make_ref_fixtures.py

`make -C oracle ref` compiles /root/reference/Youth.Source/LoggingModule/
loggingModule.c unchanged, with oracle/ref_logger_harness.c, into
oracle/_ref/ref_logger (git-ignored; SURVEY §8c: the logger is the one
reference module that compiles and links here).  The harness feeds the frames
below to the running logger over its POSIX queues in the sensor's message
format, lets the logger record them (saveFrameToFile, loggingModule.c:101-130,
end marker :224-226), plays the recording back through the logger's playback
thread (readFrameFromFile :404-444, sendMetadata :488-502, sendDataInChunks
:447-485) and captures every message it emits.

Outputs (data only, committed):
  tests/golden/ref_logger_rec.bin    the .bin the reference logger wrote
  tests/golden/ref_logger_play.msgs  u32 count; count x {u32 len, bytes}: the
                                     reference playback stream, with the header
                                     bytes the reference leaves uninitialised
                                     (ctrlCommand, filename: 32..291) zeroed

Inputs: 5 frames, numpy default_rng(0x10C6) — three 80x60 (depth 2 chunks,
colour 2 chunks), one 24x16 (1 + 1), one 97x53 (2 + 2; odd sizes); depth in
[-5, 9000) mm (negative and zero values included), random colour; frame ids
100.., timestamps 1000 + 33 k ms.  The tests re-read the frames from the
reference's recording, so no separate input file is kept.
"""
import os
import shutil
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SIZES = [(80, 60), (80, 60), (80, 60), (24, 16), (97, 53)]


def frames():
    rng = np.random.default_rng(0x10C6)
    out = []
    for k, (W, H) in enumerate(SIZES):
        d = rng.integers(-5, 9000, (H, W)).astype(np.int16)
        c = rng.integers(0, 256, (H, W, 3)).astype(np.uint8)
        out.append((100 + k, 1000 + 33 * k, d, c))
    return out


def main():
    if not os.path.isdir("/root/reference/Youth.Source"):
        sys.exit("needs /root/reference (the reference logger source)")
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_logger")
    fr = frames()
    with tempfile.TemporaryDirectory() as td:
        raw = os.path.join(td, "frames.raw")
        with open(raw, "wb") as f:
            f.write(struct.pack("<I", len(fr)))
            for fid, ts, d, c in fr:
                H, W = d.shape
                f.write(struct.pack("<4I", fid, ts, W, H))
                f.write(d.astype("<i2").tobytes())
                f.write(c.tobytes())
        rec, msgs = os.path.join(td, "rec.bin"), os.path.join(td, "play.msgs")
        r = subprocess.run([exe, raw, rec, msgs], capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            sys.exit(f"ref_logger failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
        print(r.stdout.strip().splitlines()[-1])
        shutil.copy(rec, os.path.join(HERE, "ref_logger_rec.bin"))
        shutil.copy(msgs, os.path.join(HERE, "ref_logger_play.msgs"))


if __name__ == "__main__":
    main()
