# yoda-mi355x build targets (reference Makefile: local/build/push/fmt/vet/clean)
IMAGE ?= yoda-mi355x/yoda-scheduler:0.1
PY ?= python3

.PHONY: all local native test test-gpu bench build push clean crd

all: local

# build every native artefact in-tree: C++ engine, C++ amd-smi collector, gfx950 HIP kernels
native:
	$(PY) -m yoda_scheduler_amd.ops.build

local: native
	$(PY) -c "import yoda_scheduler_amd.ops.native as n; n.core(); print('yoda-scheduler ready')"

test: native
	$(PY) -m pytest tests -q -m "not gpu"

test-gpu: native
	$(PY) -m pytest tests -q -m gpu

bench: native
	$(PY) bench.py

crd:
	$(PY) -m yoda_scheduler_amd.models.render_crd > deploy/scv-crd.yaml

build: native
	docker build . -t $(IMAGE)

push:
	docker push $(IMAGE)

clean:
	rm -f yoda_scheduler_amd/_native/*.so yoda_scheduler_amd/_native/yoda-sniffer
