"""Host-side decoding of the LeNet engine's stats rows (fedmi/engine/lenet_native.py): the device row is
lenet::Stats {float loss_sum, int correct, int count, pad} viewed as int32[4]."""
from fedmi.engine.lenet_native import LeNetNativeTrainer

import torch


def _row(loss, correct, count):
    raw = torch.zeros(4, dtype=torch.int32)
    raw[0:1].view(torch.float32)[0] = loss
    raw[1], raw[2] = correct, count
    return raw


def test_row_decodes():
    st = LeNetNativeTrainer.decode_stats(None, _row(12.5, 7, 10))
    assert (st.loss_sum, st.correct, st.count) == (12.5, 7, 10)
    assert abs(st.loss - 1.25) < 1e-9 and abs(st.acc - 70.0) < 1e-9
