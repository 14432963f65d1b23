"""Host cost of the dedisperser's plan tables on the config-4 DM list
(2026 DMs, 1024 channels, 2^20 output samples): resident MFMA plan, LDS-fed
MFMA tables, VALU offset/window tables (Dedisperser.warm builds all three)."""
import json
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from peasoup_amd import _C  # noqa: E402
sys.path.insert(0, "tools")
from baseline_configs import TSAMP, FCH1, FOFF, _dm_end_for  # noqa: E402

dm_end = _dm_end_for(2026)
dms = list(_C.generate_dm_list(0.0, dm_end, TSAMP, 64.0, FCH1, FOFF, 1024, 1.1))[:2026]
delays = _C.generate_delay_table(1024, TSAMP, FCH1, FOFF)
nsamps = (1 << 20) + _C.compute_max_delay(dms, delays) + 4096
hdr = {"source_name": "t", "tsamp": TSAMP, "fch1": FCH1, "foff": FOFF, "nchans": 1024, "nbits": 2, "nifs": 1,
       "data_type": 1, "tstart": 60000.0, "nsamples": nsamps}
torch.cuda.init()
t = time.perf_counter()
geom = _C.DedispGeometry.make(hdr, nsamps, dms, [1] * 1024)
out = {"ndm": len(dms), "geom_s": time.perf_counter() - t}
s = _C.GpuStream()
dfb = _C.DeviceFilterbank(geom, s.handle)
dd = _C.Dedisperser(dfb, s.handle)
for name, fn in (("resident_plan", lambda: dd.mfma_steps_per_channel(0, 32)),
                 ("mfma_lds_tables", lambda: dd.mfma_lds_split(0, 32)),
                 ("valu_tables", lambda: dd.choose(0, 32)),
                 ("warm_again", dd.warm)):
    t = time.perf_counter()
    fn()
    out[name + "_s"] = round(time.perf_counter() - t, 4)
print(json.dumps(out))
