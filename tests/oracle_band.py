"""The CPU oracle behind the ReuseBand interface (run_passes / halo_rows / halo_pack /
halo_unpack of a reuse-pipeline band handle), so tests drive the same multi-rank driver
(pathtracerdemo_amd/bands.py) on CPU with gloo.  TEST INFRASTRUCTURE."""
import ctypes

import numpy as np

PASS_MAP = {0: 0, 1: 11, 2: 12, 3: 3, 8: 5, 9: 6}  # include/ptx.h pass ids -> the reuse pipeline's oracle passes
GI_PASS_MAP = {1: 7, 2: 10, 8: 8, 9: 9}           # ... of a GI handle (PTX_PIPELINE_RESTIR_GI)


class OracleBand:
    def __init__(self, oracle, frame, row_begin: int, row_end: int, gi: bool = False):
        self.O, self.fr, self.b, self.e, self.gi = oracle, frame, row_begin, row_end, gi
        R = frame.reuse[0]
        self.top, self.bot = min(R, row_begin), min(R, frame.H - row_end)

    def halo_rows(self):
        return self.top, self.bot, self.fr.W * (16 + (64 if self.gi else 128))

    def run_passes(self, passes):
        fr = self.fr
        for p in passes:
            rect = (0, self.b, fr.W, self.e)
            if self.gi and p in GI_PASS_MAP:
                fr.run_gi(GI_PASS_MAP[p], threads=2, rect=rect)
                if p == 9:
                    fr.hist_valid = True
                continue
            op = PASS_MAP[p]
            if op == self.O.PASS_FINAL_REUSE:
                fr.run(op, threads=2, rect=rect, reservoir=fr.res_hist)
            else:
                fr.run(op, threads=2, rect=rect)
            if op == self.O.PASS_SPATIAL:
                fr.hist_valid = True

    def _rows(self, r0, rows, ptr, to_msg):
        if not rows:
            return
        res = self.fr.gi_res if self.gi else self.fr.reservoir
        g = self.fr.gbuffer[r0:r0 + rows]
        r = res[r0:r0 + rows]
        if to_msg:
            ctypes.memmove(ptr, g.ctypes.data, g.nbytes)
            ctypes.memmove(ptr + g.nbytes, r.ctypes.data, r.nbytes)
        else:
            gb = np.frombuffer((ctypes.c_char * g.nbytes).from_address(ptr), dtype=np.uint32).reshape(g.shape)
            rb = np.frombuffer((ctypes.c_char * r.nbytes).from_address(ptr + g.nbytes), dtype=np.uint32)
            self.fr.gbuffer[r0:r0 + rows] = gb
            res[r0:r0 + rows] = rb.reshape(r.shape)

    def halo_pack(self, top_ptr, bottom_ptr):
        self._rows(self.b, self.top, top_ptr, True)
        self._rows(self.e - self.bot, self.bot, bottom_ptr, True)

    def halo_unpack(self, top_ptr, bottom_ptr):
        self._rows(self.b - self.top, self.top, top_ptr, False)
        self._rows(self.e, self.bot, bottom_ptr, False)
