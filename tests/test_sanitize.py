"""Host sanitizer leg: the product's host sources (csrc/rt_host.cpp: scene flattening, row
bands, PPM; csrc/rt_screen.cpp: the speculative rayTraceScreen chain) and the oracle's C restatement built
with -fsanitize=address,undefined and driven by tests/sanitize/san_main.cpp on the CPU.  GPU sanitizers are
not available on this pool; the device entry points rt_screen.cpp calls are host test doubles that trace with
the oracle (tests/sanitize/san_stubs.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "sanitize")


# rt_render_screen's pipelines: the default (a continuation only behind maximum-size chunks, which these small
# frames never reach), a continuation behind every chunk (RT_SCREEN_NEXT_MIN=0: many dropped), two of them
# (RT_SCREEN_AHEAD=2: several dropped at once, buffer sets drained out of order) and none (RT_SCREEN_NEXT=0).
@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("screen_env", [{}, {"RT_SCREEN_NEXT_MIN": "0"},
                                        {"RT_SCREEN_NEXT_MIN": "0", "RT_SCREEN_AHEAD": "2"}, {"RT_SCREEN_NEXT": "0"},
                                        {"RT_SCREEN_NEXT_MIN": "0", "RT_SCREEN_PROGRESSIVE": "1"}],
                         ids=["default", "every_chunk", "ahead2", "next0", "progressive"])
def test_host_code_under_asan_ubsan(tmp_path, screen_env):
    r = subprocess.run(["make", "-C", SAN, "-j8"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1",
               **screen_env)
    r = subprocess.run([os.path.join(SAN, "_build", "san_main")], capture_output=True, text=True, timeout=600,
                       cwd=tmp_path, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize ok" in r.stdout
    assert "runtime error" not in r.stderr
