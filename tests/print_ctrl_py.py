"""Pure-Python restatement of the reference's Print_Ctrl (test infrastructure: the checker of the device output
path, include/shud_out.h).  Follows src/classes/Model_Control.cpp: Init/InitIJ (:759-858), open_file (:683-758),
PrintData (:926-960), fun_printBINARY (:893-899), fun_printASCII (:900-909)."""
import math
import struct

import numpy as np


class PrintCtrlPy:
    def __init__(self, basename, n_all, interval, iflux, start_time=0, flag_io=None, binary=True, ascii=False,
                 radiation_input_mode=0, terrain_radiation=0, solar_lonlat_mode="FORCING_FIRST", lon=0.0, lat=0.0):
        self.interval = int(interval)
        self.tau = 1440.0 if iflux else 1.0
        self.sel = np.arange(n_all) if flag_io is None else np.nonzero(np.asarray(flag_io))[0]
        self.icol = (self.sel + 1).astype(np.float64)
        self.numvar = self.sel.size
        self.buffer = np.zeros(self.numvar)
        self.num_update = 0
        header = ("# SHUD output\n"
                  f"# Radiation input mode: {'SWNET' if radiation_input_mode == 1 else 'SWDOWN'}\n"
                  f"# Terrain radiation (TSR): {'ON' if terrain_radiation else 'OFF'}\n"
                  f"# Solar lon/lat mode: {solar_lonlat_mode}\n"
                  f"# Solar lon/lat (deg): lon={lon:.6f}, lat={lat:.6f}\n").encode()
        self.fb = self.fa = None
        if binary:
            self.fb = open(str(basename) + ".dat", "wb")
            self.fb.write(header[:1023].ljust(1024, b"\0"))
            self.fb.write(struct.pack("<dd", float(start_time), float(self.numvar)))
            self.fb.write(self.icol.tobytes())
        if ascii:
            self.fa = open(str(basename) + ".csv", "w")
            self.fa.write("# Timestamp semantics: left endpoint (t-Interval)\n")
            self.fa.write(f"0\t {self.numvar}\t {int(start_time)}\n")
            for line in header.decode().splitlines()[1:]:
                self.fa.write(line + "\n")
            self.fa.write("Time_min" + "".join(f" \tX{i + 1}" for i in range(self.numvar)) + "\n")

    def print_data(self, values, t):
        self.num_update += 1
        self.buffer += np.asarray(values)[self.sel]               # buffer[i] += *(PrintVar[i]), per step
        t_floor = int(math.floor(t + 0.001))
        if t_floor % self.interval == 0:
            self.buffer *= self.tau / self.num_update
            self.num_update = 0
            tq = float(t_floor - self.interval)
            if self.fa:
                self.fa.write(f"{tq:.1f}\t" + "".join(f"{v:e}\t" for v in self.buffer) + "\n")
            if self.fb:
                self.fb.write(struct.pack("<d", tq))
                self.fb.write(self.buffer.tobytes())
            self.buffer[:] = 0.0

    def close(self):
        for f in (self.fb, self.fa):
            if f:
                f.close()
