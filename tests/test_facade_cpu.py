"""The C++ drop-in facade (include/dccrg.hpp) compiles against the C ABI and
links against libdccrgx.so and the image's MPI (no GPU needed to build):
the repo's example, every member of the class template, the plain-C header,
and the reference's own examples/game_of_life.cpp with only its include
line changed."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
MPI_INC, MPI_LIB = "/opt/conda/include", "/opt/conda/lib"
REF_EXAMPLE = "/root/reference/examples/game_of_life.cpp"


def cxx(src, out):
    from dccrg_amd import build as B

    B.build()
    return subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", INC, "-I", os.path.join(INC, "compat"), "-I",
                           MPI_INC, str(src), "-L", os.path.join(ROOT, "dccrg_amd"), "-ldccrgx",
                           os.path.join(MPI_LIB, "libmpi.so"),
                           "-Wl,-rpath," + os.path.join(ROOT, "dccrg_amd") + ":/usr/lib/x86_64-linux-gnu:" + MPI_LIB,
                           "-o", str(out)], capture_output=True, text=True)


def test_facade_example_builds(tmp_path):
    r = cxx(os.path.join(ROOT, "examples", "game_of_life.cpp"), tmp_path / "gol")
    assert r.returncode == 0, r.stderr


@pytest.mark.skipif(not os.path.exists(REF_EXAMPLE), reason="reference not present")
def test_reference_example_compiles_unchanged(tmp_path):
    """examples/game_of_life.cpp of the reference: MPI_Init, Zoltan_Initialize
    (include/compat/zoltan.h), Dccrg<game_of_life_cell> with its
    get_mpi_datatype, initialize(comm).balance_load(), the local / inner /
    outer cell ranges, cell.neighbors_of / neighbor.data, the start / wait
    halo split - only `#include "../dccrg.hpp"` becomes `#include "dccrg.hpp"`."""
    txt = open(REF_EXAMPLE).read()
    assert txt.count('#include "../dccrg.hpp"') == 1
    src = tmp_path / "game_of_life.cpp"
    src.write_text(txt.replace('#include "../dccrg.hpp"', '#include "dccrg.hpp"'))
    r = cxx(src, tmp_path / "ref_gol")
    assert r.returncode == 0, r.stderr


def test_c_header_is_plain_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "dccrgx.h"\nint main(void){ return dccrgx_abi_version() == DCCRGX_ABI_VERSION ? 0 : 1; }\n')
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", INC, str(src),
                        "-L", os.path.join(ROOT, "dccrg_amd"), "-ldccrgx",
                        f"-Wl,-rpath,{os.path.join(ROOT, 'dccrg_amd')}", "-o", str(tmp_path / "t")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert subprocess.run([str(tmp_path / "t")]).returncode == 0


def test_facade_every_member_instantiates(tmp_path):
    """Explicit instantiation compiles every member of dccrg::Dccrg (an
    unused member of a class template is otherwise never checked), with and
    without Additional_*_Items hooks (tests/advection/cell.hpp's Center and
    Is_Local shapes)."""
    src = tmp_path / "inst.cpp"
    src.write_text('''#include "dccrg.hpp"
struct Cell {
	unsigned is_alive; double x;
	std::tuple<void*, int, MPI_Datatype> get_mpi_datatype() { return std::make_tuple((void*)&x, 1, MPI_DOUBLE); }
};
struct Is_Local {
	bool is_local = false;
	template <class Grid, class Cell_Item, class Neighbor_Item>
	void update(const Grid& grid, const Cell_Item&, const Neighbor_Item& n, const int&, const Is_Local&) {
		is_local = grid.is_local(n.id);
	}
};
struct Center {
	std::array<double, 3> center;
	template <class Grid, class Cell_Item> void update(const Grid& grid, const Cell_Item& cell, const Center&) {
		center = grid.geometry.get_center(cell.id);
	}
};
template class dccrg::Dccrg<Cell, dccrg::Cartesian_Geometry>;
template class dccrg::Dccrg<Cell>;
template class dccrg::Dccrg<Cell, dccrg::Cartesian_Geometry, std::tuple<Center>, std::tuple<Is_Local>>;
// a variable-size Cell_Data (tests/variable_data_size): the serialized mode
struct Var {
	std::vector<double> v;
	std::tuple<void*, int, MPI_Datatype> get_mpi_datatype() { return std::make_tuple(v.data(), int(v.size()), MPI_DOUBLE); }
};
struct Var5 {
	std::vector<int> a;
	std::tuple<void*, int, MPI_Datatype> get_mpi_datatype(uint64_t, int, int, bool, int) {
		return std::make_tuple(a.data(), int(a.size()), MPI_INT);
	}
};
template class dccrg::Dccrg<Var>;
template class dccrg::Dccrg<Var5, dccrg::Cartesian_Geometry>;
int main() { return 0; }
''')
    r = cxx(src, tmp_path / "inst")
    assert r.returncode == 0, r.stderr


REF_KATS = ["get_cells/test1.cpp", "proc_bdy_cells/test1.cpp", "iterators/test1.cpp", "iterators/test2.cpp",
            "iterators/test3.cpp", "iterators/test4.cpp", "iterators/test5.cpp", "get_face_neighbors/test1.cpp",
            "get_neighbors_/test1.cpp", "user_neighborhood/neighbor_list_length.cpp"]


@pytest.mark.skipif(not os.path.exists("/root/reference/tests"), reason="reference not present")
@pytest.mark.parametrize("rel", REF_KATS)
def test_reference_kat_compiles(tmp_path, rel):
    """The reference's hot-path KAT programs compile against the facade with
    only the include line changed (dccrg::Types<3>, unpin_all_cells,
    get_neighborhood_of, find_neighbors_of, get_neighbors_, get_existing_cell;
    VERDICT r03 #1).  tests/test_gpu_ref_kats.py runs them."""
    txt = open(os.path.join("/root/reference/tests", rel)).read()
    txt = txt.replace('#include "../../dccrg.hpp"', '#include "dccrg.hpp"')
    src = tmp_path / "kat.cpp"
    src.write_text(txt)
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", INC, "-I", os.path.join(INC, "compat"), "-I",
                        MPI_INC, str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
