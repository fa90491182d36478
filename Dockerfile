# Runtime image: ROCm 7.2 userspace (amd-smi, HIP runtime for the gfx950 device scorer and probes),
# Python control plane, in-tree native artefacts. Default entry is the scheduler; the same image
# runs the amd-smi sniffer DaemonSet (`yoda-sniffer`).
FROM rocm/dev-ubuntu-22.04:7.2
RUN apt-get update && apt-get install -y --no-install-recommends python3-pip g++ && rm -rf /var/lib/apt/lists/*
WORKDIR /opt/yoda
COPY pyproject.toml README.md ./
COPY yoda_scheduler_amd ./yoda_scheduler_amd
COPY native ./native
RUN pip3 install --no-cache-dir pyyaml aiohttp prometheus_client pybind11 \
 && python3 -m yoda_scheduler_amd.ops.build \
 && pip3 install --no-cache-dir --no-deps .
# glibc malloc tcache for the scheduler's native threads (deploy/yoda-scheduler.yaml sets it too)
ENV GLIBC_TUNABLES=glibc.malloc.tcache_count=2048
CMD ["yoda-scheduler"]
