"""bench.py's roofline.traffic is a stored figure: the rocprofv3 FETCH_SIZE /
WRITE_SIZE summary named by bench.PMC_FILE, valid only for the kernel build it
was measured on (its kernels_sha256).  This keeps the committed summary and the
committed kernels in step: a kernel change without a new PMC pass fails here
(bench.py itself reports traffic null in that case)."""
import hashlib
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_stored_pmc_summary_matches_the_kernels():
    src = open(os.path.join(ROOT, "bench.py")).read()
    m = re.search(r'^PMC_FILE = "([^"]+)"', src, re.M)
    assert m, "bench.py names its PMC summary"
    pmc = json.load(open(os.path.join(ROOT, "profiles", m.group(1))))
    sha = hashlib.sha256(open(os.path.join(ROOT, "kwok_amd", "csrc", "kernels.hip"), "rb").read()).hexdigest()
    assert pmc["kernels_sha256"] == sha, "profiles/%s was measured on another kernels.hip" % m.group(1)
    tick = [v for k, v in pmc["kernels"].items() if "k_tick" in k]
    assert tick and tick[0]["hbm_bytes"] > 1e9  # 1M x 10M steady tick: ~1.17 GB per launch
