"""Python front end of the librsd render-graph host (include/rsd_graph.h).

It mirrors the scripting surface of Falcor's RenderGraph (RenderGraph.cpp, bound to Python
as ``falcor.RenderGraph``) that the reference's graph scripts use:

    g = RenderGraph('SVAO')
    g.create_pass('SVAO', 'SVAO', {'radius': 0.2, 'secondaryDepthMode': 'StochasticDepth', ...})
    g.add_edge('LinearizeDepth.linearDepth', 'SVAO.depth')
    g.mark_output('SVAO.ao')

plus what an application does with a graph (set_scene / compile / execute / get_output).
Every method calls the C++ host through the C ABI; errors raise ``abi.RsdError``.

``load_script`` reads a graph script WITHOUT executing it: only ``RenderGraph(...)``,
``create_pass``/``add_edge``/``mark_output`` (and the old ``addPass(createPass(...))``
spelling) with literal arguments are interpreted, via ``ast``.  ``import falcor`` (the
sibling package) provides the same names for running a script as code.
"""
from __future__ import annotations

import ast
import ctypes as C
import json
import math
from pathlib import Path

from . import abi

_FORMAT_DTYPE = {abi.FMT_R32F: ("float32", 1), abi.FMT_RG32F: ("float32", 2), abi.FMT_RGBA32F: ("float32", 4),
                 abi.FMT_R16U: ("int16", 1), abi.FMT_R8U: ("uint8", 1), abi.FMT_R8UNORM: ("uint8", 1),
                 abi.FMT_R32U: ("int32", 1), abi.FMT_R16F: ("float16", 1), abi.FMT_RG16F: ("float16", 2),
                 abi.FMT_RGBA16F: ("float16", 4), abi.FMT_RG8UNORM: ("uint8", 2)}


def _props_json(props: dict | None) -> bytes:
    out = {}
    for k, v in (props or {}).items():
        if isinstance(v, bool) or isinstance(v, (int, str)):
            out[k] = v
        elif isinstance(v, float):
            out[k] = v if math.isfinite(v) else str(v)
        elif v is None:
            out[k] = ""
        else:  # float2 / enums objects / paths: passed through by name (no hot-path pass reads them)
            out[k] = str(v)
    return json.dumps(out).encode()


def _text(fn, *args) -> str:
    need = C.c_size_t(0)
    abi.check(fn(*args, None, 0, C.byref(need)), fn.__name__)
    buf = C.create_string_buffer(need.value)
    abi.check(fn(*args, buf, need.value, C.byref(need)), fn.__name__)
    return buf.value.decode()


class PassHandle:
    """What ``create_pass`` returns (Falcor returns the RenderPass)."""

    def __init__(self, graph: "RenderGraph", name: str, type_: str, props: dict):
        self.graph, self.name, self.type, self.properties = graph, name, type_, dict(props or {})

    def __repr__(self):
        return f"<RenderPass {self.type} '{self.name}'>"


class RenderGraph:
    def __init__(self, name: str = ""):
        self.name = name
        self._L = abi.lib()
        h = C.c_void_p()
        abi.check(self._L.rsd_graph_create(name.encode(), C.byref(h)), "rsd_graph_create")
        self._h = h
        self.passes: dict[str, PassHandle] = {}
        self.edges: list[tuple[str, str]] = []
        self.outputs: list[str] = []
        self._keep = []

    # -- script surface (RenderGraph.cpp:101 createPass, :249 addEdge, :525 markOutput)
    def create_pass(self, name: str, type_: str, props: dict | None = None) -> PassHandle:
        abi.check(self._L.rsd_graph_create_pass(self._h, name.encode(), type_.encode(), _props_json(props)),
                  f"create_pass({name!r}, {type_!r})")
        self.passes[name] = PassHandle(self, name, type_, props)
        return self.passes[name]

    def add_pass(self, p: "PassDesc", name: str) -> PassHandle:  # old spelling: addPass(createPass(...), name)
        return self.create_pass(name, p.type, p.properties)

    def add_edge(self, src: str, dst: str):
        abi.check(self._L.rsd_graph_add_edge(self._h, src.encode(), dst.encode()), f"add_edge({src!r}, {dst!r})")
        self.edges.append((src, dst))

    def mark_output(self, name: str):
        abi.check(self._L.rsd_graph_mark_output(self._h, name.encode()), f"mark_output({name!r})")
        self.outputs.append(name)

    addPass, addEdge, markOutput = add_pass, add_edge, mark_output

    # -- application surface
    def set_scene(self, scene_handle, camera: abi.Camera):
        abi.check(self._L.rsd_graph_set_scene(self._h, scene_handle, C.byref(camera)), "set_scene")

    def set_input(self, name: str, ptr: int, width: int, height: int, fmt: int, layers: int = 1):
        t = abi.Texture(C.c_void_p(ptr), width, height, layers, fmt, 0)
        abi.check(self._L.rsd_graph_set_input(self._h, name.encode(), C.byref(t)), f"set_input({name!r})")

    def plan(self, width: int, height: int):
        abi.check(self._L.rsd_graph_plan(self._h, width, height), "plan")

    def compile(self, width: int, height: int, stream=None):
        abi.check(self._L.rsd_graph_compile(self._h, width, height, stream), "compile")

    def execute(self, stream=None):
        abi.check(self._L.rsd_graph_execute(self._h, stream), "execute")

    def get_output(self, name: str) -> abi.Texture:
        t = abi.Texture()
        abi.check(self._L.rsd_graph_get_output(self._h, name.encode(), C.byref(t)), f"get_output({name!r})")
        return t

    def output_tensor(self, name: str, stream=None):
        """A torch copy of a graph resource, shaped [layers][h][w][channels] (squeezed)."""
        import torch
        t = self.get_output(name)
        dt, ch = _FORMAT_DTYPE[t.format]
        out = torch.empty((t.layers, t.height, t.width, ch), dtype=getattr(torch, dt), device="cuda")
        abi.check(self._L.rsd_graph_copy_output(self._h, name.encode(), C.c_void_p(out.data_ptr()), t.bytes,
                                                stream), f"copy_output({name!r})")
        return out.squeeze(-1).squeeze(0) if t.layers == 1 else (out.squeeze(-1) if ch == 1 else out)

    def execution_order(self) -> list[str]:
        return [x for x in _text(self._L.rsd_graph_execution_order, self._h).split("\n") if x]

    def resources(self) -> dict[str, tuple[int, int, int, str]]:
        out = {}
        for line in _text(self._L.rsd_graph_resources, self._h).split("\n"):
            if line:
                key, w, h, layers, fmt = line.rsplit(" ", 4)
                out[key] = (int(w), int(h), int(layers), fmt)
        return out

    def pass_times(self) -> dict[str, float]:
        n = C.c_uint32(0)
        abi.check(self._L.rsd_graph_pass_times(self._h, None, 0, C.byref(n)), "pass_times")
        ms = (C.c_float * max(1, n.value))()
        abi.check(self._L.rsd_graph_pass_times(self._h, ms, n.value, C.byref(n)), "pass_times")
        return dict(zip(self.execution_order(), list(ms)[:n.value]))

    def dict_int(self, key: str) -> int:
        v = C.c_int64()
        abi.check(self._L.rsd_graph_get_dict_int(self._h, key.encode(), C.byref(v)), f"dict[{key!r}]")
        return v.value

    def counts(self) -> tuple[int, int]:
        p, e = C.c_uint32(), C.c_uint32()
        abi.check(self._L.rsd_graph_pass_count(self._h, C.byref(p), C.byref(e)), "pass_count")
        return p.value, e.value

    def close(self):
        if self._h:
            self._L.rsd_graph_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PassDesc:
    """``createPass(type, dict)`` of the old scripting API."""

    def __init__(self, type_: str, props: dict | None = None):
        self.type, self.properties = type_, dict(props or {})


def createPass(type_: str, props: dict | None = None) -> PassDesc:
    return PassDesc(type_, props)


def plugin_types() -> list[str]:
    return [x for x in _text(abi.lib().rsd_plugin_types).split("\n") if x]


def set_plugin_dir(path: str | Path):
    abi.check(abi.lib().rsd_plugin_set_dir(str(path).encode()), "rsd_plugin_set_dir")


# ----------------------------------------------------------------------------- script loading
class ScriptError(ValueError):
    pass


def _literal(node):
    try:
        return ast.literal_eval(node)
    except ValueError as e:
        raise ScriptError(f"line {node.lineno}: non-literal argument") from e


def load_script(source: str | Path) -> dict[str, RenderGraph]:
    """Build the graphs a graph script defines, without executing the script.

    Recognised statements (anything else is ignored): ``x = RenderGraph('name')``,
    ``x.create_pass(name, type, {...})``, ``x.add_edge(a, b)``, ``x.mark_output(n)``,
    ``x.addPass(createPass(type, {...}), name)``, ``x.addEdge``, ``x.markOutput``.
    Returns {variable name in the script: RenderGraph}; a graph built in a function and
    assigned at module level (``SVAO = render_graph_SVAO()``) appears under both names.
    """
    text = Path(source).read_text() if isinstance(source, Path) or (
        isinstance(source, str) and "\n" not in source and source.endswith(".py")) else source
    tree = ast.parse(text)
    graphs: dict[str, RenderGraph] = {}
    for node in ast.walk(tree):
        if isinstance(node, ast.Assign) and isinstance(node.value, ast.Call):
            f = node.value.func
            if isinstance(f, ast.Name) and f.id == "RenderGraph" and isinstance(node.targets[0], ast.Name):
                args = [_literal(a) for a in node.value.args]
                graphs[node.targets[0].id] = RenderGraph(*(args or [""]))
                continue
        if not (isinstance(node, ast.Expr) and isinstance(node.value, ast.Call)):
            continue
        call = node.value
        if not (isinstance(call.func, ast.Attribute) and isinstance(call.func.value, ast.Name)):
            continue
        g = graphs.get(call.func.value.id)
        if g is None:
            continue
        m = call.func.attr
        if m in ("create_pass", "add_edge", "mark_output", "addEdge", "markOutput"):
            getattr(g, m)(*[_literal(a) for a in call.args])
        elif m == "addPass":
            inner, name = call.args[0], _literal(call.args[1])
            if not (isinstance(inner, ast.Call) and isinstance(inner.func, ast.Name) and inner.func.id == "createPass"):
                raise ScriptError(f"line {node.lineno}: addPass expects createPass(...)")
            ia = [_literal(a) for a in inner.args]
            g.create_pass(name, ia[0], ia[1] if len(ia) > 1 else {})
    # `SVAO = render_graph_SVAO()` at module level: name the graph after that variable too
    returns = {}
    for fn in (n for n in tree.body if isinstance(n, ast.FunctionDef)):
        for st in ast.walk(fn):
            if isinstance(st, ast.Return) and isinstance(st.value, ast.Name) and st.value.id in graphs:
                returns[fn.name] = st.value.id
    for st in tree.body:
        if (isinstance(st, ast.Assign) and isinstance(st.value, ast.Call) and isinstance(st.value.func, ast.Name)
                and st.value.func.id in returns and isinstance(st.targets[0], ast.Name)):
            graphs[st.targets[0].id] = graphs[returns[st.value.func.id]]
    return graphs
