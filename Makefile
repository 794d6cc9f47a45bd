# Build / test / release helpers (reference Makefile: build, install, test, smoke; the
# reference's goreleaser config becomes the `release` target: version injection, one archive
# with the native components built for gfx950, and a SHA-256 checksum file).
PYTHON ?= python3
ARCH ?= gfx950
VERSION ?= $(shell $(PYTHON) -c 'import runpy; print(runpy.run_path("terraform_provider_iterative_amd/_version.py")["__version__"])')
PLUGIN_DIR ?= $(HOME)/.terraform.d/plugins/registry.terraform.io/iterative/iterative/$(VERSION)/linux_amd64
DIST ?= dist
NAME = terraform-provider-iterative-amd_$(VERSION)_linux_amd64

.PHONY: build test test-gpu bench bench-kernels install release clean

build:
	PYTORCH_ROCM_ARCH=$(ARCH) TPI_VERSION=$(VERSION) $(PYTHON) -m terraform_provider_iterative_amd._build

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
	ln -sf $(CURDIR)/bin/terraform-provider-iterative $(PLUGIN_DIR)/terraform-provider-iterative_v$(VERSION)

# make release VERSION=x.y.z: stamp the version, rebuild everything from source, archive.
release:
	sed -i 's/^__version__ = .*/__version__ = "$(VERSION)"/' terraform_provider_iterative_amd/_version.py
	PYTORCH_ROCM_ARCH=$(ARCH) $(PYTHON) -m terraform_provider_iterative_amd._build --force
	mkdir -p $(DIST)
	tar --exclude='__pycache__' --exclude='*.stamp' --transform 's,^,$(NAME)/,' -czf $(DIST)/$(NAME).tar.gz \
	    bin terraform_provider_iterative_amd README.md docs examples environment
	cd $(DIST) && sha256sum $(NAME).tar.gz > $(NAME)_SHA256SUMS

clean:
	rm -rf terraform_provider_iterative_amd/_lib $(DIST)
