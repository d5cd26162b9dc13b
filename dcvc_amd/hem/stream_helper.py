"""DCVC-HEM bitstream files, format-identical to
DCVC-HEM/src/utils/stream_helper.py (encode_i/decode_i :115-136,
encode_p/decode_p :139-160): u32 big-endian height/width, u16 q indexes,
u32 stream length, stream bytes."""
import struct
from pathlib import Path


def encode_i(height, width, q_index, bit_stream, output):
    Path(output).write_bytes(struct.pack(">2IHI", height, width, q_index, len(bit_stream)) + bytes(bit_stream))


def decode_i(inputpath):
    data = Path(inputpath).read_bytes()
    h, w, q, n = struct.unpack(">2IHI", data[:14])
    return h, w, q, data[14:14 + n]


def encode_p(string, mv_y_q_index, y_q_index, output):
    Path(output).write_bytes(struct.pack(">2HI", mv_y_q_index, y_q_index, len(string)) + bytes(string))


def decode_p(inputpath):
    data = Path(inputpath).read_bytes()
    mvq, yq, n = struct.unpack(">2HI", data[:8])
    return mvq, yq, data[8:8 + n]
