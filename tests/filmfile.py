"""Reader / writer of the reference's binary ImageFilm file ("resume" films), for tools and tests.

Layout (src/render/imagefilm.cc:1020-1075 imageFilmSave, :827-938 imageFilmLoad; strings are
written with their '\\0', src/common/file.cc:190-194): "YAF_FILMv4_0_0\\0", uint32 computer node,
uint32 base sampling offset, uint32 sampling offset, int32 width, height, cx0, cx1, cy0, cy1,
int32 number of layers, float32 weights[height][width], then per layer float32 rgba[height][width][4]
(unnormalised: sum of colour x filter weight).  Native byte order (little endian on x86-64).
The library writes these files itself (csrc/filmio.cc); this module only mirrors the format.
"""
from dataclasses import dataclass

import numpy as np

HEADER = b"YAF_FILMv4_0_0\0"


@dataclass
class Film:
    computer_node: int
    base_sampling_offset: int
    sampling_offset: int
    width: int
    height: int
    cx0: int
    cx1: int
    cy0: int
    cy1: int
    weights: np.ndarray        # (H, W) float32
    layers: list               # [(H, W, 4) float32], "combined" first

    def normalized(self, layer: int = 0):
        """Rgba::normalized (color.h:554-558): colour * (1 / weight); 0 where the weight is 0."""
        w = self.weights
        inv = np.where(w != 0, np.float32(1.0) / np.where(w != 0, w, np.float32(1)), np.float32(0)).astype(np.float32)
        return (self.layers[layer] * inv[..., None]).astype(np.float32)


def film_path(path: str, computer_node: int = 0) -> str:
    """ImageFilm::getFilmPath (imagefilm.cc:817-825)."""
    return f"{path} - node {computer_node:04d}.film"


def read(path: str) -> Film:
    with open(path, "rb") as f:
        data = f.read()
    if not data.startswith(HEADER):
        raise ValueError(f"{path}: not a YafaRay film file")
    o = len(HEADER)
    node, base, samp = np.frombuffer(data, np.uint32, 3, o).tolist()
    o += 12
    w, h, cx0, cx1, cy0, cy1, nl = np.frombuffer(data, np.int32, 7, o).tolist()
    o += 28
    weights = np.frombuffer(data, np.float32, w * h, o).reshape(h, w).copy()
    o += 4 * w * h
    layers = []
    for _ in range(nl):
        layers.append(np.frombuffer(data, np.float32, 4 * w * h, o).reshape(h, w, 4).copy())
        o += 16 * w * h
    return Film(node, base, samp, w, h, cx0, cx1, cy0, cy1, weights, layers)


def write(path: str, film: Film) -> None:
    with open(path, "wb") as f:
        f.write(HEADER)
        f.write(np.array([film.computer_node, film.base_sampling_offset, film.sampling_offset], np.uint32).tobytes())
        f.write(np.array([film.width, film.height, film.cx0, film.cx1, film.cy0, film.cy1, len(film.layers)],
                         np.int32).tobytes())
        f.write(np.ascontiguousarray(film.weights, np.float32).tobytes())
        for layer in film.layers:
            f.write(np.ascontiguousarray(layer, np.float32).tobytes())
