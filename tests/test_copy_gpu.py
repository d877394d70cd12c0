"""ured_copy_batch (csrc/copy.hip): the HIP-graph steps' batched refresh of their static inputs."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_copy_batch_units_and_sizes(dev):
    from ured_hip.ops import copy_batch
    g = torch.Generator(device=dev).manual_seed(0)
    base = torch.randint(0, 255, (4099,), device=dev, dtype=torch.uint8, generator=g)
    srcs = [torch.randn(16, 2048, 3, device=dev, generator=g),               # 16-B units
            torch.randint(-5, 5, (16, 2048), device=dev, generator=g),       # int64
            torch.randn(7, device=dev, generator=g),                         # 28 B: 4-B units
            base[1:4098],                                                    # odd offset and size: 1-B units
            torch.empty(0, device=dev)]                                      # empty: skipped
    srcs += [torch.randn(5, 3, device=dev, generator=g) for _ in range(14)]  # 19 items: two launches
    dsts = [torch.full_like(s, 7) for s in srcs]
    copy_batch(list(zip(dsts, srcs)))
    for d, s in zip(dsts, srcs):
        assert torch.equal(d, s)
    with pytest.raises(ValueError):
        copy_batch([(torch.empty(3, device=dev), torch.empty(4, device=dev))])


def test_refresh_static_unique_rows(dev):
    import numpy as np
    from ured_hip.ops import PartBounds, UniqueRows, refresh_static
    lab = np.array([[3, -1, 5, 3], [-1, -1, 2, 7]])
    lab2 = np.array([[4, -1, 1, 4], [-1, -1, 0, 6]])
    static = {"x": torch.zeros(2, 8, 3, device=dev), "src_unique": UniqueRows(lab, 10, dev, bucket=8),
              "part_bounds": PartBounds(np.zeros((2, 8)))}
    x = torch.randn(2, 8, 3, device=dev)
    batch = {"x": x, "src_unique": UniqueRows(lab2, 10, dev, bucket=8), "part_bounds": PartBounds(np.zeros((2, 8)))}
    refresh_static(static, batch)
    assert torch.equal(static["x"], x)
    for f in UniqueRows.FIELDS:
        assert torch.equal(getattr(static["src_unique"], f), getattr(batch["src_unique"], f)), f
