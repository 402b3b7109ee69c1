"""CPU test of the child script that runs the hipHostRegister cases of
tests/test_gpu_host_inplace.py: it names its cases and refuses others (exit 2)
before any device call, and the names match the GPU test's parameters."""
import os
import subprocess
import sys

import pytest

SCRIPT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_host_register_cases.py")


@pytest.mark.parametrize("argv", [[], ["nope"]])
def test_host_register_cases_usage(argv):
    r = subprocess.run([sys.executable, SCRIPT] + argv, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "registered|shorter0|shorter4" in r.stderr


def test_case_names_match_the_gpu_test():
    import ast

    here = os.path.dirname(os.path.abspath(__file__))
    src = open(os.path.join(here, "test_gpu_host_inplace.py")).read()
    assert '["registered", "shorter0", "shorter4"]' in src
    tree = ast.parse(open(SCRIPT).read())
    names = [n for n in ast.walk(tree) if isinstance(n, ast.Assign)
             and any(getattr(t, "id", None) == "CASES" for t in n.targets)]
    assert names and sorted(k.value for k in names[0].value.keys) == ["registered", "shorter0",
                                                                      "shorter4"]
