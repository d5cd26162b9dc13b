"""Bitstream files and padding helpers, format-identical to
DCVC-DC/src/utils/stream_helper.py (encode_i/decode_i :94-116,
encode_p/decode_p :119-139, get_padding_size :22-31,
get_downsampled_shape :34-37, get_state_dict :40-47)."""
import struct
from pathlib import Path

import torch


def get_padding_size(height, width, p=64):
    new_h = (height + p - 1) // p * p
    new_w = (width + p - 1) // p * p
    return 0, new_w - width, 0, new_h - height


def get_downsampled_shape(height, width, p):
    new_h = (height + p - 1) // p * p
    new_w = (width + p - 1) // p * p
    return int(new_h / p + 0.5), int(new_w / p + 0.5)


def filesize(path):
    p = Path(path)
    if not p.is_file():
        raise ValueError(f'Invalid file "{path}".')
    return p.stat().st_size


def get_state_dict(ckpt_path):
    ckpt = torch.load(ckpt_path, map_location=torch.device("cpu"), weights_only=True)
    if "state_dict" in ckpt:
        ckpt = ckpt["state_dict"]
    if "net" in ckpt:
        ckpt = ckpt["net"]
    return {(k[len("module."):] if k.startswith("module.") else k): v for k, v in ckpt.items()}


def _flag(q_in_ckpt, q_index):
    return (int(bool(q_in_ckpt)) << 7) + (int(q_index) << 1)


def pack_i(height, width, q_in_ckpt, q_index, bit_stream):
    return struct.pack(">2IBI", height, width, _flag(q_in_ckpt, q_index), len(bit_stream)) + bytes(bit_stream)


def unpack_i(data):
    h, w, flag, n = struct.unpack(">2IBI", data[:13])
    return h, w, (flag >> 7) > 0, (flag & 0x7F) >> 1, data[13:13 + n]


def pack_p(bit_stream, q_in_ckpt, q_index, frame_idx):
    return struct.pack(">BBI", _flag(q_in_ckpt, q_index), frame_idx, len(bit_stream)) + bytes(bit_stream)


def unpack_p(data):
    flag, frame_idx, n = struct.unpack(">BBI", data[:6])
    return (flag >> 7) > 0, (flag & 0x7F) >> 1, frame_idx, data[6:6 + n]


def encode_i(height, width, q_in_ckpt, q_index, bit_stream, output):
    Path(output).write_bytes(pack_i(height, width, q_in_ckpt, q_index, bit_stream))


def decode_i(inputpath):
    return unpack_i(Path(inputpath).read_bytes())


def encode_p(string, q_in_ckpt, q_index, frame_idx, output):
    Path(output).write_bytes(pack_p(string, q_in_ckpt, q_index, frame_idx))


def decode_p(inputpath):
    return unpack_p(Path(inputpath).read_bytes())
