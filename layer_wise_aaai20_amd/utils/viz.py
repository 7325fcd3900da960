"""Network-graph visualisation (``CIFAR10/core.py:343-411``) without pydot: builds Graphviz DOT
source for a dict-defined network; ``svg()`` renders through the ``dot`` binary when installed."""
from __future__ import annotations

import shutil
import subprocess
from functools import singledispatch
from inspect import signature

import numpy as np
import torch

from ..models.graph import build_graph, sep


@singledispatch
def cat(*xs):
    raise NotImplementedError(type(xs[0]))


@cat.register(torch.Tensor)
def _(*xs):
    return torch.cat(xs)


@cat.register(np.ndarray)
def _(*xs):
    return np.concatenate(xs)


@singledispatch
def to_numpy(x):
    raise NotImplementedError(type(x))


@to_numpy.register(torch.Tensor)
def _(x):
    return x.detach().cpu().numpy()


@to_numpy.register(np.ndarray)
def _(x):
    return x


class ColorMap(dict):
    palette = ("bebada,ffffb3,fb8072,8dd3c7,80b1d3,fdb462,b3de69,fccde5,bc80bd,ccebc5,ffed6f,"
               "1f78b4,33a02c,e31a1c,ff7f00,4dddf8,e66493,b07b87,4e90e3,dea05e,d0c281,f0e189,"
               "e9e8b1,e0eb71,bbd2a4,6ed641,57eb9c,3ca4d4,92d5e7,b15928").split(",")

    def __missing__(self, key):
        self[key] = self.palette[len(self) % len(self.palette)]
        return self[key]


def get_params(mod):
    return {p.name: getattr(mod, p.name, "?") for p in signature(type(mod)).parameters.values()}


class DotGraph:
    colors = ColorMap()

    def __init__(self, net, size=15, direction="LR"):
        graph = build_graph(net)
        self.nodes = [(k, {"tooltip": f"{type(n).__name__} {get_params(n)!r:.1000}",
                           "fillcolor": "#" + self.colors[type(n)]}) for k, (n, _) in graph.items()]
        self.edges = [(src, k) for k, (_, ins) in graph.items() for src in ins]
        self.size, self.direction = size, direction

    def dot_source(self) -> str:
        lines = [f'digraph G {{ rankdir={self.direction}; size="{self.size}";',
                 '  node [shape=box, style="rounded,filled", fillcolor="#ffffff"];']
        clusters = {}
        for name, attr in self.nodes:
            parts = name.split(sep)
            clusters.setdefault(tuple(parts[:-1]), []).append((name, parts[-1], attr))
        for path, nodes in clusters.items():
            if path:
                lines.append(f'  subgraph "cluster_{sep.join(path)}" {{ label="{path[-1]}"; '
                             'style="rounded,filled"; fillcolor="#77777744";')
            for name, label, attr in nodes:
                lines.append(f'    "{name}" [label="{label}", fillcolor="{attr["fillcolor"]}", '
                             f'tooltip="{attr["tooltip"].replace(chr(34), chr(39))}"];')
            if path:
                lines.append("  }")
        for a, b in self.edges:
            lines.append(f'  "{a}" -> "{b}";')
        lines.append("}")
        return "\n".join(lines)

    def svg(self) -> str:
        if shutil.which("dot") is None:
            raise RuntimeError("graphviz `dot` not installed; use dot_source()")
        return subprocess.run(["dot", "-Tsvg"], input=self.dot_source().encode(),
                              capture_output=True, check=True).stdout.decode()


def walk(dict_, key):
    while key in dict_:
        key = dict_[key]
    return key


def remove_by_type(net, node_type):
    """Drop nodes of a type (e.g. Identity) for compact pictures (core.py:407-411)."""
    graph = build_graph(net)
    remap = {k: i[0] for k, (v, i) in graph.items() if isinstance(v, node_type)}
    return {k: (v, [walk(remap, x) for x in i]) for k, (v, i) in graph.items()
            if not isinstance(v, node_type)}
