"""Helper run by tests/test_gt4py_plugin.py in a subprocess that can import the reference gt4py.

Registers gt:mi355x in the reference registry, builds each case through the REFERENCE frontend
and pipeline, and checks (1) field_info equals the reference numpy backend's, (2) the generated
library is byte-identical to the one gt4py_amd's own frontend produces for the same definition.
Prints one line per case; exits non-zero on any mismatch.
"""
import sys, types, os, importlib.util
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import gt4py.cartesian.gtscript as ref_gtscript
import gt4py_amd
import stencil_cases as sc_my
real_mod = sys.modules["gt4py_amd.gtscript"]
sys.modules["gt4py_amd.gtscript"] = ref_gtscript; gt4py_amd.gtscript = ref_gtscript
spec = importlib.util.spec_from_file_location("stencil_cases_ref", os.path.join(REPO, "tests", "stencil_cases.py"))
sc_ref = importlib.util.module_from_spec(spec); spec.loader.exec_module(sc_ref)
sys.modules["gt4py_amd.gtscript"] = real_mod; gt4py_amd.gtscript = real_mod
from gt4py_amd import gt4py_plugin
gt4py_plugin.register()
from gt4py_amd import gtscript as my
names = sys.argv[1:] or ["hdiff_f64", "hdiff_f32", "tridiag", "lap5", "copy", "vertical_advection_dycore", "suite_hdiff_weight", "native_functions", "horizontal_regions", "suite_runtime_if_nested_while", "higher_dimensional_fields", "variable_offsets_ij", "k_offset_write_backward", "lowdim_inputs", "suite_matmul", "suite_typed_temporary", "data_dim_stencil", "abs_k_literal", "abs_k_field", "abs_k_conditional", "iterator_access"]
STRICT = {"hdiff_f64", "hdiff_f32", "tridiag", "lap5", "copy", "vertical_advection_dycore", "suite_hdiff_weight",
          "higher_dimensional_fields", "variable_offsets_ij", "k_offset_write_backward", "lowdim_inputs", "suite_matmul",
          "suite_typed_temporary", "data_dim_stencil"}
bad = []
for name in names:
    case = sc_ref.CASES[name]
    s_ref = ref_gtscript.stencil(backend="gt:mi355x", definition=case.definition, externals=case.externals, name=f"plug.{name}", rebuild=True)
    try:
        s_np = ref_gtscript.stencil(backend="numpy", definition=case.definition, externals=case.externals, name=f"plugnp.{name}")
    except NotImplementedError:  # e.g. absolute K indexing: the reference numpy backend raises
        s_np = ref_gtscript.stencil(backend="debug", definition=case.definition, externals=case.externals, name=f"plugdbg.{name}")
    assert s_ref.field_info == s_np.field_info, name
    plug_path = list(gt4py_plugin._LAUNCHERS)[-1]
    mc = sc_my.CASES[name]
    s_my = my.stencil(backend="gt:mi355x", definition=mc.definition, externals=mc.externals, name=f"my.{name}")
    comp = [c.cell_contents for c in type(s_my).run.__closure__][0].compiled
    print(name, "SAME library" if plug_path == comp.lib_path else "different library")
    if plug_path != comp.lib_path and name in STRICT:
        bad.append(name)
    if plug_path != comp.lib_path:
        import difflib
        a = open(os.path.join(os.path.dirname(plug_path), "stencil.hip")).read().splitlines()
        b = comp.source.splitlines()
        d = list(difflib.unified_diff(b, a, lineterm="", n=0))
        print("\n".join(d[:30]))

if bad:
    print("MISMATCH", bad)
    sys.exit(1)
print("OK")
