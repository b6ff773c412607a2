"""The CPU parsers of untrusted bytes under hostile input:
tests/native/parser_fuzz.cpp drives cc_pcrc_decode / cc_pcrc_load (the per-page
CRC sidecar) and cc_chunk_meta_sn / cchost::ChunkFileMetaPage::decode (the chunk
metapage, chunkserver_chunkfile.cpp:90-130) with every truncation, extensions,
header bit flips, forged self-consistent headers and byte storms.  Here it runs
as a plain build; scripts/sanitize.sh runs it (and host_test's CPU cases and
this whole CPU suite) on ASan/UBSan builds.  No GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parser_fuzz_plain(tmp_path):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    lib = os.path.join(ROOT, "curve_amd")
    exe = str(tmp_path / "parser_fuzz")
    subprocess.run([cxx, "-O1", "-std=c++17", "-o", exe, os.path.join(ROOT, "tests", "native", "parser_fuzz.cpp"),
                    os.path.join(ROOT, "curve_amd", "host", "libcurvehost.a"), f"-L{lib}", "-lcurvecrc",
                    f"-Wl,-rpath,{lib}", "-lpthread"], check=True)
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "parser_fuzz: ok" in r.stdout


def test_reader_pool_under_thread_sanitizer(tmp_path):
    """cc_scan_files' persistent io threads (curve_amd/csrc/reader_pool.h) under
    ThreadSanitizer: thousands of batches of 1..24 participants, each index run
    once, each work item taken once, results visible after run() returns, pools
    torn down while idle (tests/native/reader_pool_stress.cpp).  Host only."""
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "reader_pool_stress")
    src = os.path.join(ROOT, "tests", "native", "reader_pool_stress.cpp")
    b = subprocess.run([cxx, "-O1", "-g", "-std=c++17", "-fsanitize=thread", "-o", exe, src, "-lpthread"],
                       capture_output=True, text=True)
    if b.returncode != 0 and "tsan" in (b.stderr or "").lower():
        pytest.skip("no ThreadSanitizer runtime")
    assert b.returncode == 0, b.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "reader_pool_stress: ok" in r.stdout and "ThreadSanitizer" not in r.stderr


@pytest.mark.parametrize("mode", [{}, {"CURVE_CRC_FOLD_SPLIT": "1"}, {"CURVE_CRC_FOLD_SPLIT": "0"},
                                  {"CURVE_CRC_NO_FOLD": "1"}])
def test_cpu_primitive_loops_under_address_sanitizer(tmp_path, mode):
    """Every loop of the CPU primitive (csrc/crc32c_cpu.cpp, built from source
    with ASan/UBSan) over buffers of their exact size, at each loop's edges and
    three alignments (tests/native/crc_cpu_bounds.cpp): no load past a buffer's
    end, values equal to a bitwise CRC32C.  Host only."""
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "crc_cpu_bounds")
    b = subprocess.run([cxx, "-O1", "-g", "-std=c++17", "-msse4.2", "-mpclmul", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "include"),
                        "-o", exe, os.path.join(ROOT, "curve_amd", "csrc", "crc32c_cpu.cpp"),
                        os.path.join(ROOT, "tests", "native", "crc_cpu_bounds.cpp")], capture_output=True, text=True)
    if b.returncode != 0 and "asan" in (b.stderr or "").lower():
        pytest.skip("no AddressSanitizer runtime")
    assert b.returncode == 0, b.stderr
    env = {k: v for k, v in os.environ.items() if not k.startswith("CURVE_CRC_")}
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=dict(env, **mode))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "crc_cpu_bounds: ok" in r.stdout
