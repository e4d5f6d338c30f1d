/* dccrg_cartesian_geometry.hpp - the facade's dccrg::Cartesian_Geometry lives
 * in dccrg.hpp (reference dccrg_cartesian_geometry.hpp); programs including
 * this name get it. */
#include "dccrg.hpp"
