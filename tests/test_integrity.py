"""Per-page CRC sidecar format + IntegrityService state machine (CPU parts)."""
import numpy as np
import pytest

from curve_amd import integrity as I


def test_table_roundtrip_and_corruption():
    pc = np.random.default_rng(0).integers(0, 2**32, 4096, dtype=np.uint64).astype(np.uint32)
    buf = I.encode_table(pc, 4096, chunk_sn=9)
    pb, sn, got = I.decode_table(buf)
    assert pb == 4096 and sn == 9 and (got == pc).all()
    for pos in (3, 20, 33, I.HEADER_BYTES + 7, len(buf) - 1):
        b = bytearray(buf)
        b[pos] ^= 0x01
        with pytest.raises(I.TableCorrupt):
            I.decode_table(bytes(b))
    with pytest.raises(I.TableCorrupt):
        I.decode_table(buf[:-4])


def test_service_state_machine(tmp_path):
    svc = I.IntegrityService()
    try:
        S = I.IntegrityJobState
        assert svc.PauseJob(1) == I.IntegrityOpStatus.FAILURE_UNKNOWN   # unknown job
        assert svc.ScheduleJob(1, 7, str(tmp_path)) == I.IntegrityOpStatus.SUCCESS
        assert svc.ScheduleJob(1, 7, str(tmp_path)) == I.IntegrityOpStatus.FAILURE_UNKNOWN  # duplicate id
        j = svc.wait(1, 20)
        assert j.state == S.FINISHED and j.progress == 100 and j.copyset == 7   # empty dir
        assert svc.CancelJob(1) == I.IntegrityOpStatus.FAILURE_UNKNOWN  # already finished
        assert [x.id for x in svc.ListJobs()] == [1]
        # a job can be paused before it starts, then resumed; or canceled
        svc.PauseJob(1)
        assert svc.ScheduleJob(2, 8, str(tmp_path)) == I.IntegrityOpStatus.SUCCESS
        svc.wait(2, 20)
        assert svc.ResumeJob(2) == I.IntegrityOpStatus.FAILURE_UNKNOWN  # not paused
    finally:
        svc.close()
