"""Writes tests/golden/trig_tie_inputs.npy: every finite float (|x| < 2^28 pi/2) whose fast Horner-form
Float32 sin / cos (include/srhip_math.h srm_jsin_fma / srm_jcos_fma) is flagged by srm_jtie in some
device tier -- the rows that take the device's exact re-evaluation branch (srhip_eval_impl.h
jtrigf_*).  Produced by the exhaustive checker itself (tools/check_trigf.c, SRHIP_TIE_DUMP); ~2 min
on 8 cores.  Usage: python tests/golden/make_trig_ties.py"""
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

with tempfile.TemporaryDirectory() as d:
    exe, dump = os.path.join(d, "check_trigf"), os.path.join(d, "ties.bin")
    subprocess.run(["gcc", "-O2", "-march=x86-64-v3", "-ffp-contract=off", "-fopenmp",
                    os.path.join(ROOT, "tools", "check_trigf.c"), "-lm", "-o", exe], check=True)
    subprocess.run([exe], check=True, env=dict(os.environ, SRHIP_TIE_DUMP=dump))
    bits = np.fromfile(dump, dtype=np.uint32)
np.save(os.path.join(HERE, "trig_tie_inputs.npy"), bits)
print(len(bits), "flagged inputs")
