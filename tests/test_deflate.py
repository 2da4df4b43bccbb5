"""GeoTIFF tiles encoded by the engine (csrc/kf_deflate.h, ops.kernels.TileEncoder):
predictor 3 + one fixed-Huffman zlib stream per 256 x 256 float32 tile, the
format of the reference's per-timestep DEFLATE GeoTIFFs
(observations.py:354-394).  Host runner here (the same row encoder the gfx950
kernel runs); the device streams are pinned bit-identical to it on the GPU."""
import datetime as dt
import zlib

import numpy as np
import pytest
import torch

import kafka_inferenceengine_amd as k
from kafka_inferenceengine_amd.input_output.tiff import _read_tiff_py, read_tiff, tiff_info, write_tiff_tiles
from kafka_inferenceengine_amd.ops.kernels import TileEncoder


def _planes(n, H, W, seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    out = []
    for i in range(n):
        f = np.sin(xx / (17.0 + i)) * np.cos(yy / 23.0) + 0.01 * rng.standard_normal((H, W))
        f[(yy // 40 + xx // 40) % 5 == 0] = 0.0           # flat patches: long runs
        out.append((f * (i + 1)).astype(np.float32))
    return np.stack(out)


def _pred3_tile(plane, ty, tx):
    """Predictor-3 bytes of one zero-padded 256^2 tile (TIFF TN3, little-endian samples)."""
    t = np.zeros((256, 256), np.float32)
    blk = plane[ty * 256:(ty + 1) * 256, tx * 256:(tx + 1) * 256]
    t[:blk.shape[0], :blk.shape[1]] = blk
    b = t.view(np.uint8).reshape(256, 256, 4)[:, :, ::-1]          # MSB first
    rows = np.ascontiguousarray(b.transpose(0, 2, 1)).reshape(256, 1024)
    d = rows.copy()
    d[:, 1:] = (rows[:, 1:].astype(np.int16) - rows[:, :-1].astype(np.int16)).astype(np.uint8)
    return d.tobytes()


@pytest.mark.parametrize("H,W", [(256, 256), (300, 520)])
def test_tile_streams_decode_to_predicted_bytes(H, W):
    planes = _planes(2, H, W)
    enc = TileEncoder()
    packed, sizes, offs = enc.encode(torch.from_numpy(planes.reshape(2, -1)), H, W)
    tx, ty = TileEncoder.tiles(H, W)
    assert sizes.numel() == 2 * tx * ty
    buf = packed.numpy().tobytes()
    raw_total = 0
    for i in range(sizes.numel()):
        p, t = divmod(i, tx * ty)
        stream = buf[int(offs[i]):int(offs[i]) + int(sizes[i])]
        assert stream[:2] == b"\x78\x01"
        got = zlib.decompress(stream)             # checks the Adler-32 too
        assert got == _pred3_tile(planes[p], t // tx, t % tx), i
        raw_total += len(got)
    # flat patches and smooth rows compress; fixed-Huffman worst case is 9/8
    assert int(sizes.sum()) < raw_total


def test_geotiff_from_encoded_tiles_roundtrip(tmp_path):
    H, W = 300, 520
    planes = _planes(1, H, W, seed=3)
    packed, sizes, offs = TileEncoder().encode(torch.from_numpy(planes.reshape(1, -1)), H, W)
    gt = [576452.58, 10.0, 0.0, 4324696.15, 0.0, -10.0]
    p = tmp_path / "lai_A2017001.tif"
    write_tiff_tiles(p, H, W, packed.numpy(), offs.numpy(), sizes.numpy(), gt, "EPSG:32630")
    a, info = read_tiff(p)
    assert np.array_equal(a, planes[0])
    assert info["geotransform"] == gt and info.get("epsg") == 32630
    b, _ = _read_tiff_py(p)                        # the independent Python decoder
    assert np.array_equal(b, planes[0])
    ti = tiff_info(p)
    assert ti["compression"] == 8 and ti["predictor"] == 3 and ti["tiled"] and ti["tile"] == (256, 256)


def test_single_value_and_noise_tiles():
    """Extremes of the run-length encoder: a constant tile (runs of 258 across
    the whole row) and incompressible noise (literals only, 8/9-bit codes)."""
    H = W = 256
    const = np.full((1, H * W), 0.5, np.float32)
    noise = np.random.default_rng(9).standard_normal((1, H * W)).astype(np.float32)
    for planes in (const, noise):
        packed, sizes, offs = TileEncoder().encode(torch.from_numpy(planes), H, W)
        got = zlib.decompress(packed.numpy()[:int(sizes[0])].tobytes())
        assert got == _pred3_tile(planes.reshape(H, W), 0, 0)
    assert int(TileEncoder().encode(torch.from_numpy(const), H, W)[1][0]) < 4000    # ~95 bits per row


@pytest.mark.gpu
def test_device_tile_encoder_bit_identical_to_host(cuda):
    H, W = 1100, 700
    planes = _planes(3, H, W, seed=5)
    host = TileEncoder().encode(torch.from_numpy(planes.reshape(3, -1)), H, W)
    dev = TileEncoder().encode(torch.from_numpy(planes.reshape(3, -1)).to(cuda), H, W)
    torch.cuda.synchronize()
    assert torch.equal(dev[1].cpu(), host[1]) and torch.equal(dev[2].cpu(), host[2])
    total = int(host[1].sum())
    assert torch.equal(dev[0][:total].cpu(), host[0][:total])


@pytest.mark.gpu
def test_kafka_output_device_encoder_files(cuda, tmp_path):
    """Reference-cadence output with the device encoder: every parameter's
    mean and uncertainty GeoTIFF per timestep decodes to the device rasters
    bit for bit (masked strip: the output's own mean planes)."""
    mask = np.ones((600, 520), bool)
    mask[::9] = False
    grid = [dt.datetime(2017, 1, 1) + dt.timedelta(days=16 * i) for i in range(4)]

    def run(out):
        obs = k.SyntheticBHRObservations(mask, n_train=60, device=cuda, stream=False, n_pool=2, seed=1)
        kf = k.LinearKalman(obs, out, mask, k.create_nonlinear_observation_operator, k.TIP_PARAMETERS,
                            state_propagation=k.propagate_information_filter_LAI, device=cuda)
        kf.set_trajectory_uncertainty(np.array([0, 0, 0, 0, 0, 0, 0.04]))
        kf.run(grid, kf.state_from_prior(k.JRCPrior(k.TIP_PARAMETERS, mask)), None, None)
        torch.cuda.synchronize()

    ref = k.DeviceOutput(k.TIP_PARAMETERS, keep_history=True)
    run(ref)
    out = k.KafkaOutput(k.TIP_PARAMETERS, [0, 10, 0, 0, 0, -10], "EPSG:32630", str(tmp_path), encoder="device")
    run(out)
    out.flush()
    assert out.writer_stats()["deflate_backend"].startswith("device")
    for ts, (m, u) in ref.history.items():
        for p in range(7):
            name = f"{k.TIP_PARAMETERS[p]}_{ts.strftime('A%Y%j')}"
            assert np.array_equal(read_tiff(tmp_path / f"{name}.tif")[0].reshape(-1), m[p].cpu().numpy())
            assert np.array_equal(read_tiff(tmp_path / f"{name}_unc.tif")[0].reshape(-1), u[p].cpu().numpy())
