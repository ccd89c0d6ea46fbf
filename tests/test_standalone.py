"""Standalone trainer (reference main.py train(epoch)/test(epoch)) and the
utils twins (progress bar, format_time, get_mean_and_std, init_params)."""
import io

import torch

from fedmi import ckpt
from fedmi.cli import train as train_cli
from fedmi.models import build_model
from fedmi.utils.progress import ProgressBar, format_time
from fedmi.utils.stats import get_mean_and_std, init_params


def test_standalone_train_saves_best_and_resumes(tmp_path):
    args = ["--device", "cpu", "--n-train", "512", "--n-test", "256", "--root", str(tmp_path),
            "-a", "solo", "--metrics", str(tmp_path / "m.jsonl")]
    assert train_cli.main(args + ["--epochs", "2", "--cosine", "--t-max", "4"]) == 0
    path = ckpt.client_ckpt_path(tmp_path, "solo")
    c = ckpt.load(path)
    assert set(c) == {"net", "acc", "epoch"}
    assert list(c["net"]) == list(build_model("lenet").state_dict())
    assert 0.0 < c["acc"] <= 100.0 and c["epoch"] in (0, 1)
    lines = (tmp_path / "m.jsonl").read_text().splitlines()
    assert len(lines) == 2
    # resume continues the epoch count from the checkpoint
    assert train_cli.main(args + ["--epochs", "1", "--resume"]) == 0
    assert len((tmp_path / "m.jsonl").read_text().splitlines()) == 3
    assert '"epoch": %d' % (c["epoch"] + 1) in (tmp_path / "m.jsonl").read_text().splitlines()[-1]


def test_cosine_closed_form_matches_torch():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=0.1)
    sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=10)
    for e in range(10):
        assert abs(opt.param_groups[0]["lr"] - train_cli.cosine_lr(0.1, e, 10)) < 1e-9
        opt.step()
        sch.step()


def test_format_time_two_units():
    assert format_time(0) == "0ms"
    assert format_time(0.25) == "250ms"
    assert format_time(65.5) == "1m5s"
    assert format_time(3600 + 5) == "1h5s"
    assert format_time(2 * 86400 + 3 * 3600 + 60) == "2D3h"


def test_progress_bar_without_tty():
    buf = io.StringIO()
    bar = ProgressBar(stream=buf, width=120)
    for i in range(5):
        bar.update(i, 5, "Loss: 1.000")
    out = buf.getvalue().splitlines()
    assert len(out) == 1 and out[0].endswith("5/5") and "Loss: 1.000" in out[0]


def test_mean_std_and_init_params():
    x = torch.randint(0, 256, (64, 3, 8, 8), dtype=torch.uint8)
    mean, std = get_mean_and_std(x, chunk=10)
    xf = x.double() / 255
    assert torch.allclose(mean.double(), xf.mean((0, 2, 3)), atol=1e-6)
    assert torch.allclose(std.double(), xf.flatten(2).std(2, unbiased=False).mean(0), atol=1e-6)
    m = init_params(build_model("ResNet18"))
    assert float(m.linear.bias.detach().abs().sum()) == 0.0
    assert float(m.bn1.weight.detach().min()) == 1.0
