"""Julia's Float32 sin / cos as the device evaluates them (include/srhip_math.h srm_jfn /
srm_jred_near / srm_jred_cw / srm_jtrigf_q, srhip_eval_impl.h jtrigf_rows): each of the three
per-wave tiers returns srm_jtrigf's bits for EVERY float it may see -- an exhaustive check over all
2^32 inputs (tools/check_trigf.c, ~35 s on 8 cores) -- and so does their Horner form (the device
default since round 6) on every row its tie test leaves unflagged."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_trig_tiers_exhaustive(tmp_path):
    exe = str(tmp_path / "check_trigf")
    subprocess.run(["gcc", "-O2", "-march=x86-64-v3", "-ffp-contract=off", "-fopenmp",
                    os.path.join(ROOT, "tools", "check_trigf.c"), "-lm", "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith(("cos tiers", "sin tiers"))]
    assert len(lines) == 2 and all(ln.count(" 0 wrong") == 3 for ln in lines), r.stdout
    # round 6: the Horner-form tiers -- every row srm_jtie leaves unflagged returns srm_jtrigf's bits, and
    # the flagged rows (re-evaluated exactly on the device) are a tiny share of each tier's inputs
    fast = [ln for ln in r.stdout.splitlines() if "fast tiers vs srm_jtrigf" in ln]
    assert len(fast) == 2 and all(ln.count(" / 0,") + ln.rstrip().endswith(" / 0") == 3 for ln in fast), r.stdout
    for ln in fast:
        for part in ln.split(":", 1)[1].split(","):
            n_in, flagged = int(part.split()[1]), int(part.split("inputs")[1].split("/")[0])
            assert flagged < 1e-6 * n_in, ln
