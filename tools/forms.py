"""Tool-side kernel-form selection for A/B runs: SKML_TOOL_FORMS="agg_tiles:1,dec_rows_serial:1" is
applied through skml_debug_form (the library itself reads no environment switches)."""
import os


def apply():
    from sketchml_amd import _lib
    spec = os.environ.get("SKML_TOOL_FORMS", "")
    for item in filter(None, spec.split(",")):
        name, value = item.split(":")
        _lib.lib.skml_debug_form(_lib.FORMS[name], int(value))
