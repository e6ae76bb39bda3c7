"""``falcor`` scripting names for graph scripts run as code on the librsd host.

The reference's graph scripts (``from falcor import *``; ``RenderGraph(...)``,
``create_pass``, ``add_edge``, ``mark_output``, older ``createPass``/``addPass``) resolve
to ``rsd.graph``, which builds the graph in the C++ host through include/rsd_graph.h.
``rsd.graph.load_script`` reads a script without executing it.
"""
from rsd.graph import RenderGraph, createPass, load_script, plugin_types, set_plugin_dir  # noqa: F401

__all__ = ["RenderGraph", "createPass"]
