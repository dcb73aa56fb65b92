# Convenience front end over tools/build.py (ninja + hipcc --offload-arch=gfx950).
#
# The reference builds with `make` (libpga.a via nvcc -dc) and runs its first
# example with `make test` (reference Makefile:1-23); the same verbs work here.
#
#   make              every artefact: libpga_amd/_C.so, build/libpga.{so,a}, examples, refsem
#   make lib          C API only: build/libpga.so + build/libpga.a (no torch)
#   make examples     reference examples E1-E3 (+ gen_tsp, plain-C consumers)
#   make test         CPU test suite (no GPU needed)
#   make test-gpu     GPU test suite (needs an MI355X)
#   make run-e1|run-e2|run-e3   run a reference example (GPU)
#   make bench        headline benchmark, one GPU (bench.py)
#   make clean

PYTHON ?= python
JOBS   ?= 8
BUILD  := $(PYTHON) tools/build.py -j $(JOBS)

.PHONY: all lib examples test test-gpu run-e1 run-e2 run-e3 bench clean

all:
	$(BUILD)

lib:
	$(BUILD) --no-torch build/libpga.so build/libpga.a

examples:
	$(BUILD) --no-torch build/examples/e1_onemax_float build/examples/e2_knapsack build/examples/e3_tsp \
	  build/examples/gen_tsp build/examples/onemax_bits build/examples/islands_multi_gpu

test: all
	$(PYTHON) -m pytest tests -x -q -m "not gpu"

test-gpu: all
	$(PYTHON) -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread

run-e1: examples
	build/examples/e1_onemax_float

run-e2: examples
	build/examples/e2_knapsack

run-e3: examples
	build/examples/gen_tsp | build/examples/e3_tsp

bench: all
	$(PYTHON) bench.py

clean:
	rm -rf build libpga_amd/_C.so
