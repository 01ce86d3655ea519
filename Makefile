# tensorhive_fixed_amd developer targets (reference Makefile: app/dev/dev-deps/docs/codestyle/clean)
PY ?= python

.PHONY: all build kernels native test test-gpu bench profile codestyle clean

all: build test

build: kernels native            ## gfx950 kernels (libthk.so) + native tools, in-tree
kernels:
	$(PY) -m tensorhive_fixed_amd.ops.build
native:
	$(PY) -m tensorhive_fixed_amd.native.build

test:                            ## CPU suite (what CI runs; GPU tests are skipped without a GPU)
	$(PY) -m pytest tests -x -q -m "not gpu"

test-gpu:                        ## on an MI355X box
	$(PY) -m pytest tests -x -q -m gpu

bench:                           ## flagship: Llama-3-8B bf16 train step, tokens/s JSON line
	$(PY) bench.py

profile:                         ## per-kernel time of the flagship step
	cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats -d $(CURDIR)/gpurun_out/prof -o run \
		--output-format csv -- $(PY) $(CURDIR)/bench.py --steps 2 --warmup 1

codestyle:
	$(PY) -m pyflakes tensorhive_fixed_amd tests 2>/dev/null || $(PY) -m compileall -q tensorhive_fixed_amd tests

clean:
	rm -rf tensorhive_fixed_amd/ops/_build tensorhive_fixed_amd/ops/libthk.so tensorhive_fixed_amd/native/bin \
		tensorhive_fixed_amd/native/lib .pytest_cache
