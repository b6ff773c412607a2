"""The verify-on-read access-pattern probe (diagnostic cc_page_list_probe_dev,
the ceiling cc_verify_reads_dev is held to): its host-side page list -- the
pages of a batch of reads, read after read, as CSChunkFile::Read's requests
touch them (chunkserver_chunkfile.cpp:497-536; a partly covered page counts
whole) -- against a per-read loop, its argument checks without a GPU, and on
the device its per-page words against a numpy restatement of the reduction."""
import ctypes

import numpy as np
import pytest


def test_read_pages_list_matches_a_per_read_loop():
    from curve_amd import crc as C
    rng = np.random.default_rng(31)
    for pb in (4096, 512):
        offs = rng.integers(0, 1 << 24, 300)
        lens = rng.integers(0, 40000, 300)
        lens[::17] = 0
        want = []
        for o, n in zip(offs.tolist(), lens.tolist()):
            if n:
                want.extend(range(o // pb, (o + n - 1) // pb + 1))
        got = C.read_pages_list(offs, lens, pb)
        assert got.dtype == np.int64 and got.tolist() == want
    assert C.read_pages_list([], [], 4096).size == 0


def test_page_list_probe_arguments_need_no_gpu():
    from curve_amd import _lib
    L = _lib.lib()
    buf = ctypes.c_void_p(4096)
    assert L.cc_page_list_probe_dev(None, 0, None, 0, None, None) == _lib.CC_OK  # empty list
    assert L.cc_page_list_probe_dev(None, 4096, buf, 1, buf, None) == _lib.CC_EINVAL
    assert L.cc_page_list_probe_dev(buf, 100, buf, 1, buf, None) == _lib.CC_EINVAL  # pool not whole pages
    assert L.cc_page_list_probe_dev(buf, 4096, ctypes.c_void_p(4100), 1, buf, None) == _lib.CC_EINVAL  # list alignment


@pytest.mark.gpu
def test_page_list_probe_words_on_device():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from curve_amd import crc as C
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(7)
    host = rng.integers(0, 256, 64 << 20, dtype=np.uint8)
    pool = torch.from_numpy(host).to(dev)
    for n in (1, 2, 3, 63, 64, 65, 5000, 70000):
        pages = rng.integers(0, (64 << 20) // 4096, n).astype(np.int64)
        out = torch.full((n,), 7, dtype=torch.int32, device=dev)
        C.page_list_probe(pool, torch.from_numpy(pages).to(dev), n, out)
        torch.cuda.synchronize()
        w = host.view(np.uint32).reshape(-1, 16, 64)[pages]  # [page][row j][lane]
        x = w[:, 0, :].astype(np.uint64)
        for j in range(1, 16):
            x = (((x << 1) | (x >> 31)) & 0xFFFFFFFF) ^ w[:, j, :]
        want = np.bitwise_xor.reduce(x.astype(np.uint32), axis=1)
        assert (out.cpu().numpy().view(np.uint32) == want).all(), n
    # an index past the pool reads page 0 (no access outside the pool)
    bad = torch.tensor([3, (64 << 20) // 4096, 1 << 40], dtype=torch.int64, device=dev)
    out = torch.zeros(3, dtype=torch.int32, device=dev)
    C.page_list_probe(pool, bad, 3, out)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert o[1] == o[2] and o[0] != o[1]


@pytest.mark.gpu
def test_library_loaded_before_torch_still_finds_the_device():
    """curve_amd._lib.lib() imports torch before it loads libcurvecrc, so a
    process that touches the library first still has ONE HIP runtime (torch's
    wheel loads its own libamdhip64 by path; two runtimes left libcurvecrc with
    no usable device).  A child process loads the library, then torch, then
    calls the device."""
    import os
    import subprocess
    import sys
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "load_order_probe.py"), "lib"], cwd=root,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "lib probe ok" in r.stdout and "failed" not in r.stdout, r.stdout


@pytest.mark.gpu
def test_page_list_probe_shares_the_streams_tail_block():
    """The probe's dynamic tail takes a slot set of the stream's tail block, as
    the page kernel does, and leaves the other one zero: page CRC launches
    interleaved with probe launches on one stream stay exact."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from curve_amd import crc as C
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(17)
    host = rng.integers(0, 256, 256 << 20, dtype=np.uint8)
    pool = torch.from_numpy(host).to(dev)
    want = C.page_crc(pool, 4096).clone()
    pages = torch.from_numpy(rng.integers(0, (256 << 20) // 4096, 200000).astype(np.int64)).to(dev)
    out = torch.empty(200000, dtype=torch.int32, device=dev)
    for _ in range(5):
        C.page_list_probe(pool, pages, 200000, out)
        got = C.page_crc(pool, 4096)
        C.page_list_probe(pool, pages, 200000, out)
        C.page_list_probe(pool, pages, 200000, out)
        assert torch.equal(got, want)
