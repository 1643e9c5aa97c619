python - <<'PY'
import numpy as np
rng=np.random.default_rng(0)
X=rng.random((7291,256)); y=rng.integers(0,10,7291)
with open("/tmp/usps_syn.train","w") as f:
    for i in range(7291):
        f.write(str(y[i]+1)+" "+" ".join(f"{j+1}:{X[i,j]:.6f}" for j in range(256))+"\n")
PY
for i in 1 2; do timeout -k 10 120 python -m libskylark_amd.cli.svd -k 10 --prefix /tmp/o /tmp/usps_syn.train 2>&1 | grep -v amdgpu.ids || exit 1; done
SKH_PROFILE=1 timeout -k 10 120 python -m libskylark_amd.cli.svd -k 10 --prefix /tmp/o /tmp/usps_syn.train 2>&1 | grep -v amdgpu.ids
