# Build: libsimplex.so (gfx950 kernels + C-ABI), the ./solver CLI, and the
# CPU oracle (test infrastructure).  `make -j8`.  Outputs stay in-tree (git-ignored,
# shipped to the GPU box with the snapshot).
ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
ARCH      ?= gfx950
PKG       := simplex_method_gpu_amd
SRC       := $(PKG)/csrc
BUILD     := $(PKG)/_build
HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Iinclude
LDFLAGS   := -L$(ROCM)/lib -Wl,-rpath,$(ROCM)/lib -lrccl

LIB       := $(PKG)/libsimplex.so
CLI       := solver
GLPKDRV   := solver_glpk

all: $(LIB) $(CLI) $(GLPKDRV) oracle

$(BUILD)/spx_kernels.o: $(SRC)/spx_kernels.hip $(SRC)/spx_kernels.h $(SRC)/spx_tableau.h $(SRC)/spx_tabdev.h $(SRC)/spx_device.h $(SRC)/spx_fold.h $(SRC)/spx_common.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/spx_reinv.o: $(SRC)/spx_reinv.hip $(SRC)/spx_reinv.h $(SRC)/spx_device.h $(SRC)/spx_fold.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/spx_tableau.o: $(SRC)/spx_tableau.hip $(SRC)/spx_tableau.h $(SRC)/spx_tabdev.h $(SRC)/spx_grid.h $(SRC)/spx_loop.h $(SRC)/spx_device.h $(SRC)/spx_fold.h $(SRC)/spx_common.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/spx_loop.o: $(SRC)/spx_loop.hip $(SRC)/spx_loop.h $(SRC)/spx_grid.h $(SRC)/spx_device.h $(SRC)/spx_common.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/spx_api.o: $(SRC)/spx_api.cpp $(SRC)/spx_loop.h $(SRC)/spx_kernels.h $(SRC)/spx_reinv.h $(SRC)/spx_tableau.h $(SRC)/spx_device.h include/simplex.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(BUILD)/spx_kernels.o $(BUILD)/spx_reinv.o $(BUILD)/spx_tableau.o $(BUILD)/spx_loop.o $(BUILD)/spx_api.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^ $(LDFLAGS)

$(CLI): $(SRC)/solver_main.cpp $(SRC)/lp_io.cpp $(SRC)/lp_io.h $(SRC)/mps_io.cpp $(SRC)/mps_io.h include/simplex.h $(LIB)
	g++ -O2 -std=c++17 -Wall -pthread -Iinclude -o $@ $(SRC)/solver_main.cpp $(SRC)/lp_io.cpp $(SRC)/mps_io.cpp -L$(PKG) -Wl,-rpath,'$$ORIGIN/$(PKG)' -lsimplex

# GLPK CPU-baseline counterpart (solver_glpk.cpp): libglpk bound at run time
$(GLPKDRV): $(SRC)/glpk_driver.cpp $(SRC)/lp_io.cpp $(SRC)/lp_io.h
	g++ -O2 -std=c++17 -Wall -pthread -o $@ $(SRC)/glpk_driver.cpp $(SRC)/lp_io.cpp -ldl

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD) $(LIB) $(CLI) $(GLPKDRV)
	$(MAKE) -C oracle clean

.PHONY: all clean oracle

# Experiment builds (A/B against the default: tools/pass_ab.py, tools/ab_libs.py)
# go to $(AB), which travels to the GPU box only while it exists: `make abclean`
# after the A/B.  (The product ships one libsimplex.so.)
AB        := $(PKG)/_ab

# generic experiment build: make xlib X=name XFLAGS="-DSPX_PRICE_DEEP=0"
xlib:
	@mkdir -p $(AB)/x$(X)
	$(HIPCC) $(HIPFLAGS) $(XFLAGS) -c $(SRC)/spx_kernels.hip -o $(AB)/x$(X)/spx_kernels.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(AB)/x$(X)/libsimplex.so $(AB)/x$(X)/spx_kernels.o $(BUILD)/spx_reinv.o $(BUILD)/spx_tableau.o $(BUILD)/spx_loop.o $(BUILD)/spx_api.o $(LDFLAGS)

# persistent-loop experiment build: make xloop X=name XFLAGS="-DSPX_LOOP_FU=4"
xloop:
	@mkdir -p $(AB)/l$(X)
	$(HIPCC) $(HIPFLAGS) $(XFLAGS) -c $(SRC)/spx_loop.hip -o $(AB)/l$(X)/spx_loop.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(AB)/l$(X)/libsimplex.so $(BUILD)/spx_kernels.o $(BUILD)/spx_reinv.o $(BUILD)/spx_tableau.o $(AB)/l$(X)/spx_loop.o $(BUILD)/spx_api.o $(LDFLAGS)

abclean:
	rm -rf $(AB)

.PHONY: xlib xloop abclean
