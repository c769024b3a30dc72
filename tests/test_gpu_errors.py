"""GPU error paths: a frame that fails after finish_frame (thinning that does not converge within the
launch cap) must not be served afterwards (have_frame was set before the deferred checks).
"""
import os

import pytest

import aos_gpu
import orchard

pytestmark = pytest.mark.gpu


def test_failed_frame_is_not_served(monkeypatch):
    cfg = orchard.CONFIGS["C1"]   # T ~ 13 at 0.1 m: more than one temporal block of 8 iterations
    cloud = orchard.generate(cfg)
    ctx = aos_gpu.Ctx(aos_gpu.default_params(grid_resolution=cfg.res))
    ctx.set_polygon(orchard.polygon(cfg))
    good = ctx.seedgen(cloud)   # a good frame first: the state the failure must clear
    assert good["thin_iters"] > 8
    gg = ctx.gvd_from_seedgen()
    assert len(gg["nodes"]) > 0
    monkeypatch.setenv("AOS_DEBUG_THIN_CAP", "1")   # one launch: thinning cannot converge
    with pytest.raises(RuntimeError, match="did not converge"):
        ctx.seedgen(cloud)
    for call in (ctx.gvd_from_seedgen, ctx.gvd_async):
        with pytest.raises(RuntimeError, match="no seed-gen frame"):
            call()
    with pytest.raises(RuntimeError, match="no frame"):
        ctx.debug_grid("raster", (good["height"], good["width"]))
    monkeypatch.delenv("AOS_DEBUG_THIN_CAP")
    again = ctx.seedgen(cloud)   # the handle recovers on the next good frame
    assert again["thin_iters"] == good["thin_iters"]
    assert len(ctx.gvd_from_seedgen()["nodes"]) == len(gg["nodes"])
    ctx.close()
    assert "AOS_DEBUG_THIN_CAP" not in os.environ
