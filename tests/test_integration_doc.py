"""The reference-side adapter shown in INTEGRATION.md (GpuPathTracer, the
drop-in for CUDAPathTracer / raytrace_tile) compiles against the reference's
own headers and include/ptgpu.h.  Needs /root/reference (build container)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src")) or not shutil.which("g++"),
                    reason="reference sources not present")
def test_integration_adapter_compiles_against_reference_headers(tmp_path):
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    i = doc.index("```cpp\n// src/gpu_pathtracer.h")
    j = doc.index("```", i + 6)
    (tmp_path / "gpu_pathtracer.h").write_text(doc[i + 7:j])
    (tmp_path / "check.cpp").write_text('#include "gpu_pathtracer.h"\nint main() { return 0; }\n')
    inc = [f"-I{tmp_path}", f"-I{ROOT}/include", f"-I{REF}/src", f"-I{REF}/src/static_scene",
           f"-I{REF}/CMU462/include", f"-I{REF}/CMU462/include/CMU462", f"-I{REF}/CMU462/deps/glew/include"]
    r = subprocess.run(["g++", "-std=gnu++11", "-fsyntax-only", "-w", "-DGLEW_NO_GLU"] + inc +
                       [str(tmp_path / "check.cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
