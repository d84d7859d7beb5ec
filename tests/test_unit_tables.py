"""CPU: k_emit's table-driven pod path restated on the host.
tools/micro/unit_tables_check.cpp builds the per-shape unit tables with the
engine's own builder (templates.cpp build_unit_tables) and forms every patch
as the kernel does - static bytes | 16-byte windows of the job's value row -
for 4 specs x 82 status shapes x 3 creation times, under the default template
and the custom templates of tests/templates (pod_c.tpl puts IP digits and a
creationTimestamp slot into one unit: the two-overlay case).  Every patch must
equal the spec program's assembly (pod_controller.go:404-439 over the template;
the program itself is checked against gotmpl.py in test_template_cpu.py)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_unit_tables_reproduce_the_program(tmp_path):
    exe = str(tmp_path / "unit_tables_check")
    subprocess.run(["g++", "-std=c++17", "-O1", "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "kwok_amd", "csrc"),
                    os.path.join(ROOT, "tools", "micro", "unit_tables_check.cpp"),
                    os.path.join(ROOT, "kwok_amd", "csrc", "templates.cpp"),
                    os.path.join(ROOT, "kwok_amd", "csrc", "gotemplate.cpp"), "-o", exe], check=True)
    tpls = [os.path.join(ROOT, "tests", "templates", n) for n in ("pod_a.tpl", "pod_b.tpl", "pod_c.tpl")]
    r = subprocess.run([exe] + tpls, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout, r.stdout
    two = int(r.stdout.split("mismatches, ")[1].split()[0])
    assert two > 0, "no unit with two overlays was exercised"
