"""Measurement (not product): does the order of loading libyucsum and torch matter for
torch's view of the GPU, and the library's? Each case in a fresh interpreter. (Since
round 5 yustack_amd._lib loads torch before the library; the last case loads the
library by hand, as before.)"""
import subprocess
import sys

CASES = {
    "torch first": "import torch; a=torch.cuda.is_available(); from yustack_amd import _lib; L=_lib.lib(); print(a, L.yu_device_count(), torch.cuda.is_available())",
    "lib loaded first (no call)": "from yustack_amd import _lib; L=_lib.lib(); import torch; print(torch.cuda.is_available(), L.yu_device_count())",
    "lib called first": "from yustack_amd import _lib; L=_lib.lib(); n=L.yu_device_count(); import torch; print(n, torch.cuda.is_available())",
    "ctypes load first (no torch import before)": "import ctypes; L=ctypes.CDLL('yustack_amd/libyucsum.so'); n=L.yu_device_count(); import torch; print(n, torch.cuda.is_available())",
}
for name, code in CASES.items():
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    print(f"{name}: rc={r.returncode} out={r.stdout.strip()} err={r.stderr.strip()[-200:]}", flush=True)
