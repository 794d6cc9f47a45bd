# Build / test / release helpers (reference Makefile: build, install, test, smoke).
PYTHON ?= python3
ARCH ?= gfx950
PLUGIN_DIR ?= $(HOME)/.terraform.d/plugins/registry.terraform.io/iterative/iterative/0.1.0/linux_amd64

.PHONY: build test test-gpu bench bench-kernels install clean

build:
	PYTORCH_ROCM_ARCH=$(ARCH) $(PYTHON) -m terraform_provider_iterative_amd._build

test: build
	$(PYTHON) -m pytest tests -q -m "not gpu"

test-gpu: build
	$(PYTHON) -m pytest tests -q -m gpu

bench: build
	$(PYTHON) bench.py

bench-kernels: build
	$(PYTHON) bench/bench_kernels.py

# Make the plugin discoverable by a real `terraform` (filesystem mirror layout).
install: build
	mkdir -p $(PLUGIN_DIR)
	ln -sf $(CURDIR)/bin/terraform-provider-iterative $(PLUGIN_DIR)/terraform-provider-iterative_v0.1.0

clean:
	rm -rf terraform_provider_iterative_amd/_lib
