"""Host-side decoding of the LeNet engine's stats rows (fedmi/engine/lenet_native.py).

The head path's cross-workgroup hand-off waits (csrc/kernels/lenet_kernels.hip, K12 act2 wait and K34
gradient wait) are wall-clock bounded; on a timeout the kernel sets the row's flag word and continues.
The host must refuse such a row instead of reporting stats of a step that ran on stale data.
"""
import pytest
import torch

from fedmi.engine.lenet_native import LeNetNativeTrainer


def _row(loss, correct, count, flag):
    raw = torch.zeros(4, dtype=torch.int32)
    raw[0:1].view(torch.float32)[0] = loss
    raw[1], raw[2], raw[3] = correct, count, flag
    return raw


def test_clean_row_decodes():
    st = LeNetNativeTrainer.decode_stats(None, _row(12.5, 7, 10, 0))
    assert (st.loss_sum, st.correct, st.count) == (12.5, 7, 10)


@pytest.mark.parametrize("flag,what", [(1, "K12"), (2, "K34")])
def test_handoff_timeout_flag_raises(flag, what):
    with pytest.raises(RuntimeError, match=what):
        LeNetNativeTrainer.decode_stats(None, _row(1.0, 1, 1, flag))
