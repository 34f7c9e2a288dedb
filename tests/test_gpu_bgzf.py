"""The device BGZF row writer (tfbs_batch_rows_bgzf): the rows
formatted and deflated on the GPU must decompress -- gzip checks every member's
CRC32 and length -- to exactly the rows the host formats (tfbs_batch_rows, the
text parity tests pin against the oracle and the reference fixtures), with the
same POS numbering and BGZF framing (one gzip member per block, BC extra field,
blocks of at most 64 KiB)."""
import gzip
import os
import struct

import pytest

from helpers import T, build_batch, make_regions_synth, synth_patterns

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if T.device_count() == 0:
        pytest.fail("gpu test without a visible HIP device")


def _members(data):
    """BGZF framing: (block size, uncompressed size) of every member."""
    out, i = [], 0
    while i < len(data):
        assert data[i:i + 4] == b"\x1f\x8b\x08\x04" and data[i + 12:i + 14] == b"BC", i
        bsize = struct.unpack_from("<H", data, i + 16)[0] + 1
        isize = struct.unpack_from("<I", data, i + bsize - 4)[0]
        assert bsize <= 65536 and isize <= 65280
        out.append((bsize, isize))
        i += bsize
    assert i == len(data)
    return out


def _device_rows(b, sc, chrom, min_maf=0, chunk=None, device_codes=True):
    """Rows through the device writer, chunk regions at a time (the run flow's batches);
    device_codes: the codes stay on the GPU (the run flow) or are downloaded too."""
    n = b.num_regions
    chunk = chunk or n
    parts, fake, total_rows = [], 1, 0
    for r0 in range(0, n, chunk):
        r1 = min(n, r0 + chunk)
        b.encode(sc, r0, r1, device_codes=device_codes)
        data, fake, nr, nbytes = b.rows_bgzf(sc, chrom, min_maf, fake, r0, r1)
        blocks = _members(data)
        assert sum(x[1] for x in blocks) == nbytes
        parts.append(data)
        total_rows += nr
    data = b"".join(parts)
    return gzip.decompress(data).decode(), data, total_rows


def _compare(ps, n_samples, beds, regions, chunk=None, min_maf=0, device_codes=True):
    sc = T.Scanner(ps)
    try:
        b = build_batch(ps, n_samples, beds, regions)
        b.scan(sc, reduce=True)
        want, _ = b.rows("chr1", min_maf)
        got, data, nr = _device_rows(b, sc, "chr1", min_maf, chunk, device_codes)
    finally:
        sc.close()
    assert got == want
    assert nr == want.count("\n")
    return want, data


def test_bgzf_synthetic_rows(tmp_path):
    """Synthetic regions (indels, 300 samples): rows in one call and 3 regions at a time."""
    ps, _ = synth_patterns(tmp_path, 12, 2, 102, thr=1e-3)
    beds = [("synthetic.bed", [(1000 + 400 * j, 1200 + 400 * j) for j in range(12)])]
    regions = make_regions_synth(9, 0, 12, 300, ps.max_length, 20)
    want, _ = _compare(ps, 300, beds, regions)
    assert want.count("\n") > 20
    _compare(ps, 300, beds, regions, chunk=3, device_codes=False)
    _compare(ps, 300, beds, regions, min_maf=5)


def test_bgzf_tiny_rows_many_per_block(tmp_path):
    """4 samples: rows of ~100 bytes, hundreds per block (heads dominate)."""
    ps, _ = synth_patterns(tmp_path, 30, 2, 103, thr=5e-3)
    beds = [("synthetic.bed", [(1000 + 400 * j, 1200 + 400 * j) for j in range(40)])]
    regions = make_regions_synth(11, 0, 40, 4, ps.max_length, 0)
    want, data = _compare(ps, 4, beds, regions)
    assert want.count("\n") > 100


def test_bgzf_large_rows_compress(tmp_path):
    """20 000 samples (rows of ~0.2 MB spanning several blocks): the runs and repeated
    sample texts deflate to a small fraction of the text."""
    ps, _ = synth_patterns(tmp_path, 40, 3, 104, thr=1e-4)
    n_regions = 24
    beds = [("synthetic.bed", [(1000 + 400 * j, 1200 + 400 * j) for j in range(n_regions)])]
    regions = make_regions_synth(13, 0, n_regions, 20000, ps.max_length, 0)
    want, data = _compare(ps, 20000, beds, regions)
    assert len(want) > 4 * 65280
    assert len(data) * 4 < len(want)


def test_bgzf_c3_regions_vs_host_rows(tmp_path):
    """The C3 generator (50 000 samples, 600 PWMs), 150 regions: device BGZF == host rows."""
    names = T.synth_write_pwms(str(tmp_path), 600, 3, 3)
    ps = T.parse_pwm_files(os.path.join(str(tmp_path), "pwms.txt"), os.path.join(str(tmp_path), "thr"), 1e-4, names)
    b = T.RegionBatch(ps, 50000)
    b.synth_fill(3, 0, 150, 0)
    sc = T.Scanner(ps)
    try:
        b.scan(sc, reduce=True)
        want, _ = b.rows("chr1")
        got, data, nr = _device_rows(b, sc, "chr1", chunk=64)
    finally:
        sc.close()
    assert got == want
    assert len(data) * 8 < len(want)


def test_bgzf_text_writes_meet_zeroed_lds(tmp_path, monkeypatch):
    """TFBS_BGZF_CHECK=1: the checked bgzf_wave_kernel counts every block-text LDS write
    (always an OR, fc3b823) that meets bits already set -- a byte written twice, or a
    staged text's zero padding that is not zero.  On the C3 generator's rows (runs,
    look-back matches, literals, 50 000 samples) and on a small indel set the count stays
    0 (the call fails otherwise) and the blocks inflate to the host rows."""
    monkeypatch.setenv("TFBS_BGZF_CHECK", "1")
    names = T.synth_write_pwms(str(tmp_path), 600, 3, 3)
    ps = T.parse_pwm_files(os.path.join(str(tmp_path), "pwms.txt"), os.path.join(str(tmp_path), "thr"), 1e-4, names)
    b = T.RegionBatch(ps, 50000)
    b.synth_fill(3, 200, 60, 0)
    sc = T.Scanner(ps)
    try:
        b.scan(sc, reduce=True)
        want, _ = b.rows("chr1")
        got, _, _ = _device_rows(b, sc, "chr1", chunk=64)
    finally:
        sc.close()
    assert got == want
    (tmp_path / "small").mkdir()
    ps2, _ = synth_patterns(tmp_path / "small", 40, 3, 107, thr=1e-3)
    n_regions = 40
    beds = [("synthetic.bed", [(1000 + 400 * j, 1200 + 400 * j) for j in range(n_regions)])]
    regions = make_regions_synth(19, 0, n_regions, 3000, ps2.max_length, 20)
    _compare(ps2, 3000, beds, regions)


@pytest.mark.parametrize("batch_blocks", [None, "2"])
def test_bgzf_many_pieces_one_call(tmp_path, monkeypatch, batch_blocks):
    """One call over 640 regions (the run flow's batches are 512): 8 pieces, the host
    row plan of piece j + 1 built on the helper thread into kBgSlots + 1 plan slots
    while the GPU deflates piece j; with 2 blocks per launch the call launches many
    batches, cycling the 3 block slots (each reused after its copy back,
    hipStreamWaitEvent on bg_copied).  Inflated == the host rows."""
    if batch_blocks:
        monkeypatch.setenv("TFBS_BGZF_BATCH_BLOCKS", batch_blocks)
    ps, _ = synth_patterns(tmp_path, 40, 2, 105, thr=2e-3)
    n_regions, n_samples = 640, 600
    beds = [("synthetic.bed", [(1000 + 400 * j, 1200 + 400 * j) for j in range(n_regions)])]
    regions = make_regions_synth(15, 0, n_regions, n_samples, ps.max_length, 10)
    want, data = _compare(ps, n_samples, beds, regions)
    blocks = _members(data)
    assert len(blocks) > 3 * 2 * 3  # several launches per slot when batch_blocks is 2
    assert want.count("\n") > 500


def test_bgzf_stored_blocks_inflate_to_rows(tmp_path, monkeypatch):
    """TFBS_BGZF_STORED=1: every wave-kernel block is stored (BTYPE 00) with the block's
    text as the kernel assembled it for the CRC -- the path incompressible blocks take --
    so the members inflate (and pass gzip's CRC check) to exactly the host rows."""
    monkeypatch.setenv("TFBS_BGZF_STORED", "1")
    ps, _ = synth_patterns(tmp_path, 40, 3, 106, thr=1e-4)
    n_regions = 12
    beds = [("synthetic.bed", [(1000 + 400 * j, 1200 + 400 * j) for j in range(n_regions)])]
    regions = make_regions_synth(17, 0, n_regions, 5000, ps.max_length, 10)
    want, data = _compare(ps, 5000, beds, regions)
    blocks = _members(data)
    assert len(blocks) > 2
    assert sum(b[0] for b in blocks) > len(want)  # stored: no smaller than the text
