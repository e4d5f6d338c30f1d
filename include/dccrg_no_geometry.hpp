/* dccrg_no_geometry.hpp - the facade's dccrg::No_Geometry lives in dccrg.hpp
 * (reference dccrg_no_geometry.hpp); programs including this name get it. */
#include "dccrg.hpp"
