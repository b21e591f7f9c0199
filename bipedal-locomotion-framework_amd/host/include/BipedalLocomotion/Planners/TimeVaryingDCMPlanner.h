/**
 * @file TimeVaryingDCMPlanner.h
 * Batched receding-horizon DCM planner (TimeVaryingDCMPlanner, absent from the reference
 * snapshot), exposed through the reference's Advanceable surface
 * (src/System/include/BipedalLocomotion/System/Advanceable.h:24-46).
 *
 * Each advance():
 *   1. for every problem b and knot k = 0..N, t_k = (start + k) dt, finds the contact phase with
 *      begin <= t_k < end in that problem's ContactPhaseList and collects the corners
 *      pose * (+-L/2, +-W/2, 0) of its active contacts (the rectangle convention of
 *      ContinuousContactModel.h:32-36); r_ref_k = xi_ref_k = their centroid;
 *   2. builds every support polygon's H-rep on the device (blf_hull2d_hrep);
 *   3. solves all QPs on the device (blf_dcm_mpc_solve, include/blf/blf_c.h);
 *   4. publishes the plan (get()), then moves the window one knot forward, taking the planned
 *      xi_1 as the next initial DCM.
 * isValid() is true iff a plan exists and every problem's status is BLF_QP_SOLVED.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_PLANNERS_TIME_VARYING_DCM_PLANNER_H
#define BLF_BIPEDAL_LOCOMOTION_PLANNERS_TIME_VARYING_DCM_PLANNER_H

#include <array>
#include <cstdint>
#include <memory>
#include <vector>

#include <BipedalLocomotion/ParametersHandler/IParametersHandler.h>
#include <BipedalLocomotion/Planners/ContactPhaseList.h>
#include <BipedalLocomotion/System/Advanceable.h>
#include <blf/device.h>

namespace BipedalLocomotion
{
namespace Planners
{

struct DCMPlanBatch
{
    int batch{0};
    int horizon{0};
    double initialTime{0.0};
    std::vector<double> dcm;          /**< [batch][horizon+1][2] */
    std::vector<double> vrp;          /**< [batch][horizon][2]   */
    std::vector<int32_t> status;      /**< [batch] BLF_QP_*      */
    std::vector<int32_t> iterations;  /**< [batch]               */
};

class TimeVaryingDCMPlanner : public System::Advanceable<DCMPlanBatch>
{
    blf_dcm_mpc_params m_params{};
    double m_gravity{9.81};
    double m_footLength{0.12};
    double m_footWidth{0.09};
    int m_start{0};
    bool m_valid{false};
    std::vector<ContactPhaseList> m_plans;
    std::vector<double> m_xi0;       /**< [batch][2] */
    std::vector<double> m_height;    /**< [batch][horizon] CoM height per knot (empty: 0.53) */
    DCMPlanBatch m_output;

    blf::DeviceBuffer<double> m_dCorners, m_dXi0, m_dOmega, m_dXiRef, m_dVrpRef, m_dA, m_dB;
    blf::DeviceBuffer<double> m_dXi, m_dVrp;
    blf::DeviceBuffer<int32_t> m_dNCorners, m_dNf, m_dStatus, m_dIters;

public:
    TimeVaryingDCMPlanner();

    /**
     * Keys (all optional): "horizon" (int), "sampling_time", "gravity", "foot_length",
     * "foot_width", "dcm_weight", "vrp_weight", "terminal_weight" (scalar or 2-vector),
     * "tolerance" (tol_mu), "max_iterations" (int).
     */
    bool initialize(std::weak_ptr<ParametersHandler::IParametersHandler> handler);

    /** One footstep plan per problem (the batch size). */
    bool setContactPhaseLists(const std::vector<ContactPhaseList>& plans);
    /** Initial DCM per problem ([batch][2]). */
    bool setInitialDCM(const std::vector<std::array<double, 2>>& xi0);
    /** CoM height per problem and knot ([batch][horizon]); omega_k = sqrt(g / z_k). */
    bool setCoMHeights(const std::vector<double>& heights);

    const DCMPlanBatch& get() const final { return m_output; }
    bool isValid() const final { return m_valid; }
    bool advance() final;

    const blf_dcm_mpc_params& parameters() const { return m_params; }
    int currentKnot() const { return m_start; }
};

} // namespace Planners
} // namespace BipedalLocomotion

#endif
