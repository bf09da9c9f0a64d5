% aiyagari_egm_gpu.m -- host script for the MI355X solver (SURVEY.md §8(b) B6), the EGM model of
% Aiyagari_EGM.m.
%
% Calibration, bisection and reporting stay in MATLAB/Octave; the two inner loops are one
% gateway call each:
%   * the EGM policy iteration (Aiyagari_EGM.m:74-110, GE copy :176-212) -> aiy_egm_solve_mex
%   * the Monte-Carlo capital path (:130-155, GE copy :221-240)      -> aiy_sim_capital_mex
% The reference's GE loop sets r = r_guess inside the EGM loop (:180) but never recomputes the
% wage: every GE solve uses the w of r = 0.04 (:61).  That quirk is kept below (w_stale), so the
% bisection trace is the script's.
% Build the gateways first (aiyagari-replication_amd/mex/Makefile header, or
%   mex -I../../include -L.. -laiyagari_hip <gateway>.c   /   mkoctfile --mex ...).

clear; clc;

% ---------------------------------------------------------------- calibration (:7-56)
beta = 0.96; sigma = 5; alpha = 0.36; delta = 0.08; b = 0;
rho = 0.75; sigma_e = 0.75; N = 7; Na = 400; tol = 1e-5; max_iter = 1000; T = 10000;
use_step_gateways = false;   % true: keep the script's own while loop, one gateway call per step

l_grid = ((1:N) - 4) * sigma_e;
edges = [-Inf, ((1:N-1) - 3.5) * sigma_e, Inf];
sd = sigma_e * sqrt(1 - rho^2);
P = zeros(N, N);
for i = 1:N
    for j = 1:N
        P(i, j) = integral(@(x) normpdf(x, rho * l_grid(i), sd), edges(j), edges(j + 1));
    end
end
A = [P' - eye(N); ones(1, N)];
pi_stat = A \ [zeros(N, 1); 1];
s = exp(l_grid);
labor = s * pi_stat;

wmin = (1 - alpha) * (alpha / ((1 / beta - 1) + delta))^(alpha / (1 - alpha));
amin = min(b, wmin * s(1));
kmax = delta^(1 / (alpha - 1));
amax = kmax^alpha + (1 - delta) * kmax;
a_grid = amin + (amax - amin) * (linspace(0, 1, Na).^2)';   % column, as in :56

kdemand = @(r) labor * (alpha / (r + delta))^(1 / (1 - alpha));

% ---------------------------------------------------------------- initial solve at r = 0.04
r = 0.04;
w = (1 - alpha) * (alpha / (r + delta))^(alpha / (1 - alpha));   % :61
w_stale = w;                                 % the GE loop below never updates it (:180)
policy_c = repmat((1 + r) * a_grid + w * mean(s), 1, N);          % :64, Na x N
tic;
if use_step_gateways
    % the reference's loop (:74-110) with its body (:75-107) swapped for the gateway
    dist = 1; iter = 0;
    while dist > tol && iter < max_iter
        iter = iter + 1;
        [policy_c_next, policy_k, dist] = aiy_egm_step_mex(policy_c, a_grid, s, P, r, w, beta, ...
                                                           sigma, amin);
        policy_c = policy_c_next;
    end
else
    [policy_c, policy_k, dist, iter] = ...
        aiy_egm_solve_mex(policy_c, a_grid, s, P, r, w, beta, sigma, amin, tol, max_iter);
end
fprintf('r = %.4f: %d iterations, dist %.3e\n', r, iter, dist);

z1 = randi(N);                               % :127-128
k1 = a_grid(randi(Na));
% policy_k is Na x N here (layout 0); one rand per step (:132)
[K_s, sim_k, sim_z] = aiy_sim_capital_mex(policy_k, a_grid, P, z1, k1, rand(T - 1, 1), 0);
fprintf('K_s = %.6f\n', K_s);

% ---------------------------------------------------------------- bisection on r (:157-253)
r_low = -0.05; r_high = 1 / beta - 1;
max_r_iter = 10; r_tol = 1e-5;
r_history = zeros(max_r_iter, 1); k_supply = zeros(max_r_iter, 1); k_demand = zeros(max_r_iter, 1);
for r_iter = 1:max_r_iter
    r = (r_low + r_high) / 2;
    % warm start from the previous policy_c (the script's loop state), stale wage
    [policy_c, policy_k, dist, iter] = ...
        aiy_egm_solve_mex(policy_c, a_grid, s, P, r, w_stale, beta, sigma, amin, tol, max_iter);
    [K_s, sim_k, sim_z] = aiy_sim_capital_mex(policy_k, a_grid, P, z1, k1, rand(T - 1, 1), 0);
    K_d = kdemand(r);
    r_history(r_iter) = r; k_supply(r_iter) = K_s; k_demand(r_iter) = K_d;
    fprintf('step %2d: r = %.6f, K_s = %.6f, K_d = %.6f (%d iterations)\n', r_iter, r, K_s, ...
            K_d, iter);
    if abs(K_s - K_d) < r_tol
        break;
    elseif K_s > K_d
        r_high = r;
    else
        r_low = r;
    end
end
fprintf('equilibrium r = %.10f after %.3f s\n', r, toc);

% ---------------------------------------------------------------- the script's reporting paths
% sim_c / sim_y / sim_s of :143-148 at the last step, from the returned paths
sim_c = zeros(T, 1); sim_y = zeros(T, 1); sim_s = zeros(T, 1);
for t = 2:T
    sim_c(t) = interp1(a_grid, policy_c(:, sim_z(t)), sim_k(t - 1), 'linear', 'extrap');
    sim_y(t) = r * sim_k(t) + w_stale * s(sim_z(t));
    sim_s(t) = sim_y(t) + delta * sim_k(t) - sim_c(t);
end
sorted_k = sort(sim_k);
lorenz_k = cumsum(sorted_k) / sum(sorted_k);
gini_k = 1 - 2 * trapz((1:T) / T, lorenz_k);
fprintf('Gini coefficient for wealth: %.4f\n', gini_k);
