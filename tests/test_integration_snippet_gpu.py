"""INTEGRATION.md section 2's ctypes snippet runs as written (the binding a maintainer
would copy): it packs layer4.0.conv2's weights and runs its bf16 forward through the C ABI;
the output is checked against a torch conv of the same bf16 operands (one bf16 rounding)."""
import os
import re

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_integration_ctypes_snippet(monkeypatch):
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## 2. C ABI"):]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    monkeypatch.chdir(ROOT)
    env = {}
    exec(compile(code, "INTEGRATION.md#2", "exec"), env)
    torch.cuda.synchronize()
    x, w, y = env["x"], env["w"], env["y"]
    ref = torch.nn.functional.conv3d(x.float(), w.to(torch.bfloat16).float(), padding=4,
                                     dilation=4)
    err = (y.float() - ref).abs()
    assert (err <= 2 ** -7 * ref.abs() + 1e-3 * ref.abs().max()).all(), err.max().item()
